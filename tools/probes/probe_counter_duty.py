#!/usr/bin/env python3
"""Experiment: does stopping the rocprofiler-sdk counting context
between the service's 100 Hz reads stop the runtime's busy-polling thread?

Each mode runs in a fresh process (the context is configured before HIP starts): the
node service's sampling (amd-smi 10 Hz, device counters 100 Hz on the native sampler
threads) for --seconds, then reports the process's CPU-s/s (all threads), the busiest
threads, the counter read p50 / p99 (µs, as the sampler times them: start + read + wait +
read + stop in duty mode) and the counter rows' HBM / gfx-busy means (duty mode rates
cover only the duty window).

    python tools/probes/probe_counter_duty.py --modes 0,200,1000 --seconds 10
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(seconds: float) -> dict:
    sys.path.insert(0, ROOT)
    from rocmdash.runtime import native

    native.load()
    ok, status = native.enable_counters()
    import numpy as np

    from rocmdash.config import SamplerConfig
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.threads import thread_cpu

    agent = GpuAgent(0, cfg=SamplerConfig(smi_hz=10.0, counter_hz=100.0))
    time.sleep(1.0)
    agent.start()
    time.sleep(1.0)  # settle
    a, c0, t0 = thread_cpu(), time.process_time(), time.perf_counter()
    h0 = agent.ctr_ring.head if agent.ctr_ring is not None else 0
    time.sleep(seconds)
    b, c1, t1 = thread_cpu(), time.process_time(), time.perf_counter()
    h1 = agent.ctr_ring.head if agent.ctr_ring is not None else 0
    st = agent.sampler_stats()
    rows, _ = agent.ctr_ring.window(min(h1 - h0, 4096)) if agent.ctr_ring is not None else (np.zeros((0, 5)), None)
    agent.close()
    wall = t1 - t0
    busy = sorted(((b[t][1] - a.get(t, (b[t][0], b[t][1], 0))[1]) / wall, b[t][0]) for t in b)[::-1][:4]
    return {"counters": ok, "status": status, "duty_us": int(os.environ.get("ROCMDASH_COUNTER_DUTY_US", "0")),
            "cpu_s_per_s": round((c1 - c0) / wall, 4), "busiest_threads": [[n, round(r, 3)] for r, n in busy],
            "counter_rows_per_s": round((h1 - h0) / wall, 1),
            "counter_read_p50_us": round(st[1]["p50_us"], 1) if len(st) > 1 else None,
            "counter_read_p99_us": round(st[1]["p99_us"], 1) if len(st) > 1 else None,
            "counter_failures": int(st[1]["failures"]) if len(st) > 1 else None,
            "row_means": [round(float(x), 3) for x in np.nanmean(rows, axis=0)] if len(rows) else None}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--modes", default="0,200,1000")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        print(json.dumps(child(args.seconds)), flush=True)
        return 0
    for m in args.modes.split(","):
        env = dict(os.environ, ROCMDASH_COUNTER_DUTY_US=m)
        res = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--seconds", str(args.seconds)],
                             env=env, capture_output=True, text=True, timeout=args.seconds + 120)
        line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
        print(line[-1] if line else json.dumps({"duty_us": m, "error": res.stderr[-800:]}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
