"""Scan B's phase clocks (LongWindowSet.set_phase_clocks) in the steady incremental state:
2^24 x (8 + 4) series, 100 new rows per refresh, normal or telemetry data. Per phase
(counts + partials, gather, select, outputs) the median over refreshes of the slowest
workgroup's time from its own start to that phase, in shader-clock cycles (s_memtime,
100 MHz on CDNA: 1 cycle = 10 ns).

    python tools/probes/lw_phase_clocks.py [--shape normal] [--window 16777216]
"""

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="normal")
    ap.add_argument("--window", type=int, default=1 << 24)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--unfused", action="store_true", help="incremental pass B as its own kernel (not inside scan B)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from rocmdash.runtime import native

    nat = native.load()
    nat.set_pinned_host_rings(True)
    W = args.window
    cap = min(W, 1 << 20)
    rings = [nat.SeriesRing(8, cap), nat.SeriesRing(4, cap)]
    lw = nat.LongWindowSet(W, 0)
    lw.fused_passb = not args.unfused
    for r in rings:
        lw.add_ring(r)
    out = torch.empty((12, 8), device="cuda")
    rng = np.random.default_rng(0)
    if args.shape == "telemetry":
        blocks = [rng.integers(40, 56, (cap, 8)).astype(np.float32), rng.integers(700, 760, (cap, 4)).astype(np.float32)]
    else:
        blocks = [rng.normal(50, 10, (cap, 8)).astype(np.float32), rng.normal(500, 100, (cap, 4)).astype(np.float32)]
    stream = torch.cuda.current_stream().cuda_stream
    t = 0
    while t < W:
        for ring, b in zip(rings, blocks):
            ring.push_many(b, np.arange(t, t + cap, dtype=np.uint64))
        t += cap
        lw.refresh(out.data_ptr(), stream)
    torch.cuda.synchronize()
    lw.set_phase_clocks(True)
    phases = []
    for i in range(args.iters + 5):
        o = (t * 7919) % (cap - 100)
        for ring, b in zip(rings, blocks):
            ring.push_many(b[o:o + 100], np.arange(t, t + 100, dtype=np.uint64))
        t += 100
        lw.refresh(out.data_ptr(), stream)
        torch.cuda.synchronize()
        c = np.array(lw.phase_clocks(), dtype=np.uint64).reshape(12, 3, 8).astype(np.int64)
        if i < 5:
            continue
        # shader clocks are per XCD: every workgroup's phases against its OWN start
        start = c[:, :, 0]
        rec = {}
        for k, name in ((6, "fused_passb"), (1, "counts_partials"), (2, "to_select"), (3, "gather"), (4, "select"),
                        (5, "outputs")):
            ok = (c[:, :, k] > 0) & (start > 0)
            if ok.any():
                rec[name] = int((c[:, :, k] - start)[ok].max())
        phases.append(rec)
    keys = sorted({k for p in phases for k in p})
    med = {k: statistics.median(p[k] for p in phases if k in p) for k in keys}
    st = lw.bracket_state(0)
    print(json.dumps({"shape": args.shape, "window": W, "fused_passb": lw.fused_passb, "chunk_plan": lw.chunk_plan,
                      "cin_by_series": [x["cin"] for x in st], "exact": [[d == 0.0 for d in x["delta"]] for x in st],
                      "cycles_since_first_start_p50": med, "stats": lw.stats()}), flush=True)


if __name__ == "__main__":
    main()
