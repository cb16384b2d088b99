"""Shared by the supervisor tests on the CPU (tests/test_supervisor.py) and the GPU
(tests/test_gpu_multirank.py): start a supervised node service and watch its /metrics."""

import os
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


from rocmdash.runtime.nodemeasure import free_port, get, start_node, stop_node  # noqa: E402,F401


def scrape(port):
    """{"ts": refresh time, "gpus": set of gpu_ids on the dashboard, "up": {gpu: 0/1},
    "down": {gpu: reason}, "restarts": {gpu: n}, "stale": {(gpu, source): v}, "epoch"}
    or None."""
    from rocmdash.prom.exposition import parse_text

    code, body = get(f"http://127.0.0.1:{port}/metrics")
    if code != 200 or not body:
        return None
    out = {"ts": None, "gpus": set(), "up": {}, "down": {}, "restarts": {}, "stale": {}, "epoch": None}
    for s in parse_text(body):
        d = s.label_dict()
        if s.name == "rocmdash_node_refresh_timestamp_seconds":
            out["ts"] = s.value
        elif s.name == "amd_gpu_gfx_activity":
            out["gpus"].add(d["gpu_id"])
        elif s.name == "rocmdash_gpu_up":
            out["up"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_gpu_down_info":
            out["down"][d["gpu_id"]] = d["reason"]
        elif s.name == "rocmdash_gpu_restarts_total":
            out["restarts"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_source_stale":
            out["stale"][(d["gpu_id"], d["source"])] = s.value
        elif s.name == "rocmdash_node_epoch":
            out["epoch"] = s.value
    return out if out["ts"] is not None else None


def watch(port, until, timeout, poll_s=0.1, health=True):
    """Scrape until ``until(history)`` is true; returns the history of distinct refreshes
    [(ts, scrape)] and the /healthz codes seen."""
    hist, codes = [], []
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        s = scrape(port)
        if s is not None and (not hist or s["ts"] != hist[-1][0]):
            hist.append((s["ts"], s))
        if health and hist:  # from the first refresh on (before it the port may not listen yet)
            codes.append(get(f"http://127.0.0.1:{port}/healthz")[0])
        if hist and until(hist):
            return hist, codes
        time.sleep(poll_s)
    raise AssertionError(f"condition not reached within {timeout} s; last scrape: {hist[-1] if hist else None}")


def outage_s(hist, full: set, partial: set):
    """Seconds between the last refresh that showed every GPU in ``full`` and the first
    later refresh that showed exactly ``partial`` (the node serving without the lost GPU)."""
    last_full = None
    for ts, s in hist:
        if s["gpus"] == full:
            last_full = ts
        elif s["gpus"] == partial and last_full is not None:
            return ts - last_full
    return None


def max_gap_s(hist):
    ts = [t for t, _ in hist]
    return max((b - a for a, b in zip(ts, ts[1:])), default=0.0)
