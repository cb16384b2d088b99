#!/usr/bin/env python3
"""Host time of each piece of one N = 1 host-out refresh (NodePipeline.step), to find
the Python plumbing around the ~14 us of launch + kernel + completion flag
(tools/probes/probe_refresh_flag.py). Wraps the pipeline's and agent's methods with
perf_counter brackets; prints p50 us per piece.

    python tools/probes/probe_step_overhead.py [--steps 3000]
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
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--rccl", action="store_true", help="one-rank RCCL group + forced collective (the N > 1 path)")
    args = ap.parse_args()
    from rocmdash.runtime import native

    native.load()
    native.enable_counters()
    import torch  # noqa: F401

    from rocmdash.config import SamplerConfig
    from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.pipeline import NodePipeline

    env = dist_env_from_environ(prefer_gpu=True, world1_group=args.rccl)
    agent = GpuAgent(env.local_rank, cfg=SamplerConfig(window=4096, ring_capacity=16384), use_gpu=True)
    agg = NodeAggregator(force_collective=args.rccl)
    pipe = NodePipeline(agent, agg, prefetch=True)
    agent.prefill(4096)
    acc: dict = {}

    def wrap(obj, name):
        f = getattr(obj, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            r = f(*a, **k)
            acc.setdefault(name, []).append((time.perf_counter() - t0) * 1e6)
            return r

        setattr(obj, name, g)

    for n in ("wait_sample", "request_sample", "refresh", "wait_refresh"):
        wrap(agent, n)
    for n in ("sample_phase", "gather", "_to_host", "render_payload"):
        wrap(pipe, n)
    wrap(agg, "all_gather")
    steps = []
    for i in range(args.steps):
        t0 = time.perf_counter()
        pipe.step()
        steps.append((time.perf_counter() - t0) * 1e6)
    out = {k: round(statistics.median(v[200:]), 2) for k, v in acc.items()}
    out["step"] = round(statistics.median(steps[200:]), 2)
    print(json.dumps(out), flush=True)
    agent.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
