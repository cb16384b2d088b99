#!/usr/bin/env python3
"""Where the host-observed time of one host-out refresh goes (one MI355X):

  launch  = host time of the refresh call (Python -> native -> hipLaunchKernel), direct
            binding vs GpuAgent.refresh (adds the torch stream lookup and checks)
  wait    = launch return -> completion flag seen in mapped host memory
  kernel  = the kernel's own duration is in rocprofv3 (7.4 us, profiles/r02)

    python tools/probes/probe_refresh_flag.py [--iters 2000]
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    args = ap.parse_args()
    import numpy as np

    from rocmdash.runtime import native

    nat = native.load()
    import torch

    nat.set_pinned_host_rings(True)
    W = 4096
    rings = [nat.SeriesRing(11, 4 * W), nat.SeriesRing(4, 4 * W)]
    dws = nat.DeviceWindowSet(W, 0)
    for r in rings:
        dws.add_ring(r)
    out = torch.empty((15, 8), dtype=torch.float32, pin_memory=True)
    stream = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(0)
    t = 0

    def push(k):
        nonlocal t
        for _ in range(k):
            t += 1
            rings[0].push(rng.integers(0, 400, 11).astype(np.float32), t)
            rings[1].push(rng.integers(0, 400, 4).astype(np.float32), t)

    push(W)
    seq = dws.refresh(out.data_ptr(), stream)
    torch.cuda.synchronize()
    res = {}
    for mode in ("direct", "stream_lookup", "sync"):
        launch, wait = [], []
        for i in range(args.iters):
            push(1)
            t0 = time.perf_counter()
            if mode == "stream_lookup":
                s = torch.cuda.current_stream(0).cuda_stream
                seq = dws.refresh(out.data_ptr(), s)
            else:
                seq = dws.refresh(out.data_ptr(), stream)
            t1 = time.perf_counter()
            if mode == "sync":
                torch.cuda.current_stream(0).synchronize()
                ok = True
            else:
                ok = dws.wait_done(seq, 1.0)
            t2 = time.perf_counter()
            if not ok:
                raise SystemExit(f"no flag for refresh {i}")
            if i >= 100:
                launch.append((t1 - t0) * 1e6)
                wait.append((t2 - t1) * 1e6)
        res[mode] = {"launch_p50_us": round(statistics.median(launch), 2),
                     "wait_p50_us": round(statistics.median(wait), 2),
                     "wait_p90_us": round(sorted(wait)[int(0.9 * len(wait))], 2)}
        print(json.dumps({mode: res[mode]}), flush=True)
    torch.cuda.synchronize()
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
