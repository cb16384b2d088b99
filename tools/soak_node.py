#!/usr/bin/env python3
"""Soak of the SUPERVISED node service - the DaemonSet's entrypoint as deployed
(``rocmdash.launch`` -> supervisor + node counter process with one lane per GPU + one
rank per GPU), with a long window and node-wide window statistics - for minutes.

    python tools/soak_node.py [--seconds 240] [--window 1048576] [--refresh-hz 10] [--out soak.json]

Scrapes the supervisor's ``/metrics`` and ``/healthz`` every ``--every`` seconds and checks:

  * the node refresh timestamp advances at every scrape, ``/healthz`` answers 200;
  * every GPU's counter lane stays up (``rocmdash_counter_source_up`` 1, no stall, lane
    generation 0) and delivers ~the counter rate (``rocmdash_sampler_samples_total``);
  * no epoch change after the first (nobody lost, nobody restarted);
  * every process's own device memory (``rocmdash_node_process_device_memory_bytes``,
    DRM fdinfo) is flat after the first minute, and the node's PSS grows by at most
    ``--pss-slack-mib`` from the first minute to the end.

Prints a progress line per scrape and a JSON verdict last (exit 1 when a check fails)."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def scrape(port: int) -> dict | None:
    from rocmdash.prom.exposition import parse_text
    from rocmdash.runtime.nodemeasure import get

    code, body = get(f"http://127.0.0.1:{port}/metrics", timeout=5.0)
    if code != 200:
        return None
    out = {"ts": None, "up": {}, "stalls": {}, "lane": {}, "rows": {}, "epoch": None, "dev": {}, "pss": None,
           "gpus": set()}
    for s in parse_text(body):
        d = s.label_dict()
        if s.name == "rocmdash_node_refresh_timestamp_seconds":
            out["ts"] = s.value
        elif s.name == "rocmdash_counter_source_up":
            out["up"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_counter_source_stalls_total":
            out["stalls"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_counter_source_lane":
            out["lane"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_sampler_samples_total" and d.get("source") == "counter":
            out["rows"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_node_epoch":
            out["epoch"] = s.value
        elif s.name == "rocmdash_node_process_device_memory_bytes":
            out["dev"][f"{d['process']}:{d.get('gpu_id', '')}:{d.get('bdf', '')}"] = s.value
        elif s.name == "rocmdash_node_pss_bytes":
            out["pss"] = s.value
        elif s.name == "amd_gpu_gfx_activity":
            out["gpus"].add(d["gpu_id"])
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--seconds", type=float, default=240.0)
    ap.add_argument("--every", type=float, default=5.0)
    ap.add_argument("--window", type=int, default=1 << 20)
    ap.add_argument("--refresh-hz", type=float, default=10.0)
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--pss-slack-mib", type=float, default=32.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from rocmdash.runtime.nodemeasure import free_port, get, start_node, stop_node

    port = free_port()
    p = start_node(args.nproc, port, cpu=False, counter_daemon="on", restart_base_s=5.0,
                   env={"ROCMDASH_WINDOW": str(args.window), "ROCMDASH_COUNTER_HZ": "100", "ROCMDASH_SMI_HZ": "10"},
                   serve_args=("--refresh-hz", str(args.refresh_hz), "--node-window", "--collective-timeout", "30"))
    hist, codes, fails = [], [], []
    t0 = time.monotonic()
    try:
        while time.monotonic() - t0 < 240:  # start-up: every GPU on the dashboard with counter rows
            s = scrape(port)
            if s and len(s["gpus"]) == args.nproc and s["rows"] and min(s["rows"].values()) > 200:
                break
            if p.poll() is not None:
                raise SystemExit(f"the node service exited with {p.returncode} during start-up")
            time.sleep(1.0)
        else:
            raise SystemExit("the node service did not come up within 240 s")
        t_start = time.monotonic()
        while time.monotonic() - t_start < args.seconds:
            time.sleep(args.every)
            s = scrape(port)
            code = get(f"http://127.0.0.1:{port}/healthz", timeout=5.0)[0]
            codes.append(code)
            if s is None:
                fails.append(f"{time.monotonic() - t_start:.0f} s: /metrics did not answer")
                continue
            s["t"] = time.monotonic() - t_start
            if hist:
                a = hist[-1]
                if not (s["ts"] and a["ts"] and s["ts"] > a["ts"]):
                    fails.append(f"{s['t']:.0f} s: the node refresh did not advance")
                dt = s["t"] - a["t"]
                rates = {g: (s["rows"].get(g, 0) - a["rows"].get(g, 0)) / dt for g in s["rows"]}
                s["rates"] = rates
                if any(not (70 < r < 130) for r in rates.values()):
                    fails.append(f"{s['t']:.0f} s: counter rows/s {rates}")
            if any(v != 1.0 for v in s["up"].values()) or any(v for v in s["stalls"].values()) \
                    or any(v for v in s["lane"].values()):
                fails.append(f"{s['t']:.0f} s: a counter lane stalled: up {s['up']} stalls {s['stalls']} lane {s['lane']}")
            if code != 200:
                fails.append(f"{s['t']:.0f} s: /healthz {code}")
            hist.append(s)
            print(json.dumps({"t": round(s["t"], 1), "epoch": s["epoch"], "healthz": code,
                              "rates": {g: round(v, 1) for g, v in (s.get("rates") or {}).items()},
                              "pss_mib": round((s["pss"] or 0) / 2**20, 1),
                              "dev_mib": {k: round(v / 2**20, 1) for k, v in s["dev"].items()}}), flush=True)
    finally:
        rc = stop_node(p)
    # after the first minute: device memory flat, PSS bounded, one epoch
    late = [h for h in hist if h["t"] >= 60.0]
    if late:
        first, last = late[0], late[-1]
        for k, v in last["dev"].items():
            if k in first["dev"] and abs(v - first["dev"][k]) > 1 << 20:
                fails.append(f"device memory of {k} moved: {first['dev'][k] / 2**20:.1f} -> {v / 2**20:.1f} MiB")
        if first["pss"] and last["pss"] and last["pss"] - first["pss"] > args.pss_slack_mib * 2**20:
            fails.append(f"node PSS grew {(last['pss'] - first['pss']) / 2**20:.1f} MiB after the first minute")
    epochs = sorted({h["epoch"] for h in hist if h["epoch"] is not None})
    if len(epochs) > 1:
        fails.append(f"membership changed: epochs {epochs}")
    res = {"ok": not fails and rc == 0, "seconds": args.seconds, "window": args.window, "refresh_hz": args.refresh_hz,
           "nproc": args.nproc, "scrapes": len(hist), "healthz": sorted(set(codes)), "epochs": epochs, "rc": rc,
           "pss_mib_first_last": [round((late[0]["pss"] or 0) / 2**20, 1), round((late[-1]["pss"] or 0) / 2**20, 1)]
           if late else None,
           "dev_mib_last": {k: round(v / 2**20, 1) for k, v in (hist[-1]["dev"] if hist else {}).items()},
           "failures": fails[:20]}
    print(json.dumps(res), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
