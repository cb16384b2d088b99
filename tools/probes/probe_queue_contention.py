"""What ONE hardware queue costs the stats stage while a long-window radix chain runs
(the supervisor starts every node process with GPU_MAX_HW_QUEUES=1).

    GPU_MAX_HW_QUEUES=1 python tools/probes/probe_queue_contention.py [--window 16777216]

A LongWindowSet of W samples x 12 series with bracket mode OFF (every refresh is the full
radix chain: what a bracket miss costs) runs on stream A; the window-stats kernel of a
16-series x 4096-sample window (the service's stats stage) is launched on stream B
right behind each chain, and again with stream A idle. HIP events on stream B bracket
the stats launch: on one hardware queue both streams feed the same queue, so the stats
kernel waits for the chain ahead of it; with several queues it runs beside it. The
events on stream B only start when its queue reaches them (on one queue: after the
chain), so the host's wait from the stats launch to its completion is reported too - the
latency the service's stats stage sees. Prints one JSON line: both (p50 / p90) idle vs
behind a chain, the chain's own time, and the queue setting."""

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=1 << 24)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    import numpy as np
    import torch

    from rocmdash.runtime import native

    nat = native.load()
    nat.set_pinned_host_rings(True)
    W = args.window
    cap = min(W, 1 << 20)
    rings = [nat.SeriesRing(w, cap) for w in (8, 4)]
    lw = nat.LongWindowSet(W, 0, False)
    lw.brackets = False  # every refresh takes the radix chain (a bracket miss)
    for r in rings:
        lw.add_ring(r)
    rng = np.random.default_rng(0)
    blocks = [rng.normal(50, 10, (cap, 8)).astype(np.float32), rng.normal(500, 100, (cap, 4)).astype(np.float32)]
    a = torch.cuda.Stream()
    b = torch.cuda.Stream()
    out_lw = torch.empty((12, 8), device="cuda")
    t = 0
    while t < W:
        for ring, blk in zip(rings, blocks):
            ring.push_many(blk, np.arange(t, t + cap, dtype=np.uint64))
        t += cap
        lw.refresh(out_lw.data_ptr(), a.cuda_stream)
    torch.cuda.synchronize()
    # the stats stage: the window-stats kernel over a time-major [4096, 16] ring
    S, n = 16, 4096
    ring = torch.randn((n, S), device="cuda")
    out = torch.empty((S, 8), device="cuda")
    cols = list(range(S))

    def stats():
        nat.window_stats_raw(ring.data_ptr(), n, S, n - 1, n, cols, out.data_ptr(), b.cuda_stream, 50.0, 90.0, 99.0)

    def one(behind: bool):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if behind:
            for ring_, blk in zip(rings, blocks):
                ring_.push_many(blk[:100], np.arange(0, 100, dtype=np.uint64) + one.t)
            one.t += 100
            c0.record(a)
            lw.refresh(out_lw.data_ptr(), a.cuda_stream)
            c1.record(a)
        h0 = time.perf_counter()
        e0.record(b)
        stats()
        e1.record(b)
        e1.synchronize()  # the host's wait for the stats stage (what the service's refresh sees)
        host = (time.perf_counter() - h0) * 1e6
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3, (c0.elapsed_time(c1) * 1e3 if behind else None), host

    one.t = t
    for _ in range(5):
        one(False)
        one(True)
    idle, behind, chain, host_idle, host_behind = [], [], [], [], []
    for _ in range(args.iters):
        s_us, _, h_us = one(False)
        idle.append(s_us)
        host_idle.append(h_us)
        s_us, c_us, h_us = one(True)
        behind.append(s_us)
        chain.append(c_us)
        host_behind.append(h_us)

    def q(v):
        v = sorted(v)
        return {"p50": round(statistics.median(v), 1), "p90": round(v[int(0.9 * len(v))], 1), "max": round(v[-1], 1)}

    print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "(default 4)"), "window": W,
                      "stats_stage_us_idle": q(idle), "stats_stage_us_behind_chain": q(behind),
                      "host_wait_us_idle": q(host_idle), "host_wait_us_behind_chain": q(host_behind),
                      "chain_us": q(chain), "iters": args.iters}), flush=True)


if __name__ == "__main__":
    main()
