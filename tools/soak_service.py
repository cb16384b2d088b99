#!/usr/bin/env python3
"""Soak test of the node service: does the exporter stay flat and healthy over minutes?

Starts ``rocmdash.serve`` (world 1, live sources at the production rates: amd-smi 10 Hz,
device counters 100 Hz; node refresh at ``--refresh-hz``, 10 Hz by default = 10x the
DaemonSet's, with the node window) and scrapes its ``/metrics`` and ``/healthz`` every
``--every`` seconds for ``--seconds``. Checks, per GPU:

  * every counter the exporter calls a counter only goes up
    (``rocmdash_self_cpu_seconds_total``, ``rocmdash_sampler_samples_total`` /
    ``_failures_total`` / ``_overruns_total``, ``rocmdash_exporter_scrapes_total``);
  * ``rocmdash_node_refresh_timestamp_seconds`` advances at every scrape and
    ``/healthz`` answers 200 throughout;
  * HBM (``rocmdash_self_hbm_bytes``) does not move after start-up, and resident host
    memory (``rocmdash_self_rss_bytes``) grows by at most ``--rss-slack-mib`` from the
    first minute to the end (no leak per refresh / scrape);
  * the samplers keep their rates (samples per second of wall time).

Prints one progress line per scrape and a JSON verdict last (exit 1 when a check fails).

    python tools/soak_service.py [--seconds 240] [--refresh-hz 10] [--out soak.json]
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.error
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

COUNTERS = ("rocmdash_self_cpu_seconds_total", "rocmdash_sampler_samples_total", "rocmdash_sampler_failures_total",
            "rocmdash_sampler_overruns_total", "rocmdash_exporter_scrapes_total")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scrape(base: str) -> dict:
    from rocmdash.prom.exposition import parse_text

    with urllib.request.urlopen(base + "/metrics", timeout=5) as r:
        body = r.read().decode()
    out = {}
    for smp in parse_text(body):
        if smp.name.startswith(("rocmdash_self_", "rocmdash_sampler_", "rocmdash_exporter_scrapes",
                                "rocmdash_node_refresh_timestamp")):
            out[(smp.name, tuple(sorted(smp.label_dict().items())))] = smp.value
    return out


def _healthz(base: str) -> int:
    try:
        with urllib.request.urlopen(base + "/healthz", timeout=5) as r:
            return r.status
    except urllib.error.HTTPError as e:
        return e.code


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--seconds", type=float, default=240.0)
    ap.add_argument("--every", type=float, default=5.0)
    ap.add_argument("--refresh-hz", type=float, default=10.0)
    ap.add_argument("--source", default="auto")
    ap.add_argument("--counters", default="auto")
    ap.add_argument("--rss-slack-mib", type=float, default=16.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)

    port = _free_port()
    cmd = [sys.executable, "-m", "rocmdash.serve", "--host", "127.0.0.1", "--port", str(port), "--refresh-hz",
           str(args.refresh_hz), "--source", args.source, "--counters", args.counters, "--node-window"]
    env = dict(os.environ, PYTHONPATH=ROOT, ROCMDASH_SMI_HZ="10", ROCMDASH_COUNTER_HZ="100")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    log_path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"soak_serve_{port}.log")
    log = open(log_path, "w")
    t_start = time.monotonic()
    proc = subprocess.Popen(cmd, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT, env=env, start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    samples, failures = [], []
    try:
        deadline = time.monotonic() + 240
        while True:  # wait until the service is ready: footprint rows out, /healthz 200
            if proc.poll() is not None:
                raise RuntimeError(f"service exited with {proc.returncode} (log: {log_path})")
            if time.monotonic() > deadline:
                raise RuntimeError("service not ready within 240 s")
            try:
                if any(k[0] == "rocmdash_self_rss_bytes" for k in _scrape(base)) and _healthz(base) == 200:
                    break
            except OSError:
                pass
            time.sleep(0.5)
        t_ready = time.monotonic() - t_start
        t0 = time.monotonic()
        while True:
            t = time.monotonic() - t0
            m, hz = _scrape(base), _healthz(base)
            samples.append((t, m, hz))
            rss = max(v for k, v in m.items() if k[0] == "rocmdash_self_rss_bytes") / 2**20
            hbm = max((v for k, v in m.items() if k[0] == "rocmdash_self_hbm_bytes"), default=float("nan")) / 2**20
            ts = max(v for k, v in m.items() if k[0] == "rocmdash_node_refresh_timestamp_seconds")
            print(f"[soak] t={t:6.1f}s healthz={hz} rss={rss:.1f}MiB hbm={hbm:.1f}MiB refresh_age={time.time() - ts:.3f}s",
                  flush=True)
            if t >= args.seconds or proc.poll() is not None:
                break
            time.sleep(args.every)
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()
        log.close()

    def series(name):
        keys = sorted({k for _, m, _ in samples for k in m if k[0] == name})
        return {k: [(t, m.get(k)) for t, m, _ in samples] for k in keys}

    for name in COUNTERS:
        for k, pts in series(name).items():
            vals = [v for _, v in pts if v is not None]
            if any(b < a for a, b in zip(vals, vals[1:])):
                failures.append(f"counter went down: {k}")
    ts = [max(v for k, v in m.items() if k[0] == "rocmdash_node_refresh_timestamp_seconds") for _, m, _ in samples]
    if any(b <= a for a, b in zip(ts, ts[1:])):
        failures.append("node refresh timestamp did not advance between two scrapes")
    if any(hz != 200 for _, _, hz in samples):
        failures.append(f"/healthz not 200: {sorted({hz for _, _, hz in samples})}")
    per_gpu = {}
    for k, pts in series("rocmdash_self_rss_bytes").items():
        gid = dict(k[1]).get("gpu_id")
        after_1min = [v for t, v in pts if t >= min(60.0, args.seconds / 2) and v is not None]
        growth = (after_1min[-1] - after_1min[0]) / 2**20 if len(after_1min) > 1 else 0.0
        hbm = [v for _, v in series("rocmdash_self_hbm_bytes").get(("rocmdash_self_hbm_bytes", k[1]), []) if v is not None]
        rates = {}
        for sk, spts in series("rocmdash_sampler_samples_total").items():
            d = dict(sk[1])
            if d.get("gpu_id") == gid:
                (ta, va), (tb, vb) = spts[0], spts[-1]
                rates[d.get("source", "?")] = round((vb - va) / (tb - ta), 1) if tb > ta else None
        per_gpu[gid] = {"rss_mib_first": round(pts[0][1] / 2**20, 1), "rss_mib_last": round(pts[-1][1] / 2**20, 1),
                        "rss_growth_mib_after_1min": round(growth, 2),
                        "hbm_mib_min_max": [round(min(hbm) / 2**20, 1), round(max(hbm) / 2**20, 1)] if hbm else None,
                        "sampler_rate_hz": rates}
        if growth > args.rss_slack_mib:
            failures.append(f"gpu {gid}: RSS grew {growth:.1f} MiB after the first minute")
        if hbm and max(hbm) != min(hbm):
            failures.append(f"gpu {gid}: HBM moved {min(hbm)} -> {max(hbm)}")
    res = {"ok": not failures, "failures": failures, "seconds": round(samples[-1][0], 1), "scrapes": len(samples),
           "ready_s": round(t_ready, 2),
           "refresh_hz": args.refresh_hz, "rates": "amd-smi 10 Hz, counters 100 Hz, node window", "per_gpu": per_gpu}
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0 if not failures else 1


if __name__ == "__main__":
    raise SystemExit(main())
