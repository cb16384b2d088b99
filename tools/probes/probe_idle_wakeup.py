#!/usr/bin/env python3
"""Is a kernel's HIP-event time longer when the GPU idled before it? The node service
refreshes at 1-10 Hz, so its stats kernel starts on a GPU that idled 100 ms-1 s; the
bench's side run launches it back to back. For idle gaps of 0 / 1 / 10 / 100 ms this
times, with HIP events right around the launch: the window-stats refresh (the service's
stats stage) and a 2 µs one-wave spin kernel (no memory traffic), plus the host time of
the launch call itself (perf_counter around it).

    python tools/probes/probe_idle_wakeup.py [--reps 30]
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
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    from rocmdash.runtime import native

    nat = native.load()
    import torch

    from rocmdash.config import SamplerConfig
    from rocmdash.runtime.agent import GpuAgent

    agent = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=4096, ring_capacity=16384))
    agent.prefill(4200)
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for gap in (0.0, 0.001, 0.01, 0.1):
        out = {"idle_gap_ms": gap * 1e3}
        for name in ("stats_refresh", "spin_2us"):
            dev, host = [], []
            for i in range(args.reps + 3):
                agent.sample()
                torch.cuda.synchronize()
                time.sleep(gap)
                e0.record(stream)
                t0 = time.perf_counter()
                if name == "stats_refresh":
                    agent.refresh()
                else:
                    nat.spin(1, 2.0, stream.cuda_stream)
                t1 = time.perf_counter()
                e1.record(stream)
                e1.synchronize()
                if i >= 3:
                    dev.append(e0.elapsed_time(e1) * 1e3)
                    host.append((t1 - t0) * 1e6)
            out[name] = {"device_us_p50": round(statistics.median(dev), 2), "device_us_p90": round(sorted(dev)[int(0.9 * len(dev))], 2),
                         "launch_host_us_p50": round(statistics.median(host), 2)}
        print(json.dumps(out), flush=True)
    agent.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
