"""Probe: how much a lockstep N-rank refresh would lose to the slowest rank's read.

At N > 1 every refresh ends in one all-gather, so the node refreshes at the pace of the
slowest rank's sample: the step takes max over ranks of (counter read, SMU read). With
the per-read durations of one real GPU (``Sampler.recent_us``, csrc/sampler.cpp) this
draws N independent ranks from the measured per-step distribution and reports the
expected step read time at N = 1/2/4/8 - the efficiency the 8-GPU weak-scaling run would
lose to read tails if ranks were independent (box-wide slow phases are correlated, which
lowers the loss).

    python tools/probes/probe_lockstep_tail.py [--steps 4000] [--out f.json]
"""

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from rocmdash.runtime import native

    native.load()
    native.enable_counters()
    import torch

    from rocmdash.config import SamplerConfig
    from rocmdash.parallel.node import NodeAggregator
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.pipeline import NodePipeline

    torch.cuda.set_device(0)
    agent = GpuAgent(0, cfg=SamplerConfig(window=4096, ring_capacity=16384))
    pipe = NodePipeline(agent, NodeAggregator(), prefetch=True)
    agent.prefill(4096)
    for _ in range(100):
        pipe.step()
    agent.wait_sample()
    chunk = 900  # < the samplers' 1024 recent durations
    reads = {s.source.kind: [] for s in agent.samplers}
    done = 0
    while done < args.steps:
        k = min(chunk, args.steps - done)
        for _ in range(k):
            pipe.step()
        agent.wait_sample()
        for s in agent.samplers:
            reads[s.source.kind].extend(list(s.recent_us())[-k:])
        done += k
    agent.close()
    kinds = sorted(reads)
    arr = {k: np.asarray(v, dtype=np.float64) for k, v in reads.items()}
    n = min(len(v) for v in arr.values())
    step = np.max(np.stack([arr[k][:n] for k in kinds]), axis=0)  # both sources read concurrently
    rng = np.random.default_rng(0)
    q = lambda v: {p: round(float(np.percentile(v, p)), 2) for p in (50, 90, 99)} | {"mean": round(float(v.mean()), 2)}
    out = {"steps": int(n), "read_us": {k: q(arr[k]) for k in kinds}, "step_read_us": q(step), "lockstep": {}}
    base = float(step.mean())
    for world in (1, 2, 4, 8):
        draws = rng.choice(step, size=(200000, world)).max(axis=1)
        out["lockstep"][str(world)] = {"mean_step_read_us": round(float(draws.mean()), 2),
                                       "efficiency_vs_1": round(base / float(draws.mean()), 4)}
    # the same with every rank's wait for its read bounded at 1.5 x the median read
    cap = 1.5 * float(np.median(step))
    out["bounded_wait_cap_us"] = round(cap, 2)
    for world in (2, 4, 8):
        draws = np.minimum(rng.choice(step, size=(200000, world)), cap).max(axis=1)
        out["lockstep"][str(world)]["bounded_mean_step_read_us"] = round(float(draws.mean()), 2)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
