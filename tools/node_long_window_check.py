#!/usr/bin/env python3
"""Node-wide long-window statistics on real GPUs: the distributed radix select
(``LongWindowSet.refresh_node``, csrc/long_window.hip) against the fp64 reference of the
UNION of every rank's window.

Run under torchrun (ROCMDASH_OVERSUBSCRIBE=1 on a box with fewer GPUs than ranks):

    ROCMDASH_OVERSUBSCRIBE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \\
        --master-addr 127.0.0.1 --master-port 29561 tools/node_long_window_check.py --window 1048576

Every rank owns two rings (8 + 4 series) behind one HBM-resident LongWindowSet and pushes
rows generated from a seed of its own; every rank can therefore rebuild every other
rank's window locally and check the node statistics without moving any window. The
refreshes alternate local ``refresh`` (staging) and collective ``refresh_node`` so the
pass-0 prediction runs on mixed (local / node) state, with fills, small pushes (<= 256
rows: predicted digits) and larger ones (no prediction), then a steady stream of 100-row
pushes where node bracket mode (one record all-gather per refresh) should hit. Each node
refresh's collective steps are timed with HIP events. Rank 0 prints one JSON line; exit 0 only if
every rank matched on every node refresh.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WIDTHS = (8, 4)


def rows_for(rank: int, step: int, k: int, t0: int):
    import numpy as np

    rng = np.random.default_rng(1000 * rank + step)
    out = []
    for w in WIDTHS:
        x = rng.integers(0, 50, size=(k, w)).astype(np.float32)  # telemetry-like ties
        x[:, 0] = rng.normal(100 + 10 * rank, 20, k)  # continuous, per-rank offset
        x[:, 1] = 42.0 + rank  # a constant that differs per rank
        if w > 4:
            x[:, 2] = rng.choice(np.array([-0.0, 0.0, -1.5, 3.25], np.float32), k)
            x[:, 3] = rng.standard_cauchy(k) * 1e5
        x[rng.random((k, w)) < 0.03] = np.nan
        x[:, -1] = t0 + np.arange(k, dtype=np.float32) + rank * 0.5  # monotone
        out.append(x)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--window", type=int, default=1 << 20)
    ap.add_argument("--capacity", type=int, default=1 << 17)
    ap.add_argument("--no-brackets", action="store_true", help="radix chain on every node refresh")
    ap.add_argument("--node-fused", action="store_true",
                    help="the records' kernel streams short work lists itself (LongWindowSet.node_fused_passb)")
    ap.add_argument("--steady", type=int, default=24, help="node refreshes of 100-row pushes at the end (bracket hits)")
    args = ap.parse_args(argv)

    from rocmdash.runtime import native

    nat = native.load()
    import numpy as np
    import torch

    from rocmdash.ops.window_stats import window_stats_reference
    from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ, oversubscribed

    env = dist_env_from_environ(prefer_gpu=True, timeout_s=300, world1_group=True)
    rank, world = env.rank, env.world_size
    dev = env.device
    agg = NodeAggregator(force_collective=world == 1)
    errors = []
    if not agg.enable_native(dev):
        errors.append(f"rank {rank}: native communicator unavailable: {agg.native_error}")
    comm = agg.native.comm if agg.native is not None else None

    W, cap = args.window, args.capacity
    nat.set_pinned_host_rings(True)
    rings = [nat.SeriesRing(w, cap) for w in WIDTHS]
    lw = nat.LongWindowSet(W, dev.index)
    if args.no_brackets:
        lw.brackets = False
    if args.node_fused:
        lw.node_fused_passb = True
    for r in rings:
        lw.add_ring(r)
    S = sum(WIDTHS)
    out = torch.empty((S, 8), dtype=torch.float32, device=dev)
    # mirrors of EVERY rank's pushes (regenerated from the seeds): the union reference
    mirrors = [[np.zeros((0, w), np.float32) for w in WIDTHS] for _ in range(world)]
    plan = []
    left = W + 3
    while left > 0:  # fill in chunks the host ring holds
        k = min(cap, left)
        plan.append(("local", k))
        left -= k
    plan += [("node", 0), ("node", 100), ("node", 3), ("local", 7), ("node", 256), ("node", 1000), ("node", 0),
             ("node", cap), ("node", 64)] + [("node", 100)] * args.steady
    coll_us = []
    checks = 0
    t = 0
    node_s = []
    rec_bytes = []  # this rank's all-gathered bracket records per node refresh (0: none)
    for step, (kind, k) in enumerate(plan):
        for q in range(world):
            xs = rows_for(q, step, k, t)
            for i, x in enumerate(xs):
                mirrors[q][i] = np.concatenate([mirrors[q][i], x])[-W:]
                if q == rank:
                    rings[i].push_many(x, np.arange(t, t + k, dtype=np.uint64))
        t += k
        stream = torch.cuda.current_stream(dev).cuda_stream
        if kind == "local":
            lw.refresh(out.data_ptr(), stream)
            torch.cuda.synchronize(dev)
            continue
        rb0 = lw.stats()["node_record_bytes"]
        t0 = time.perf_counter()
        lw.refresh_node(out.data_ptr(), stream, 50.0, 90.0, 99.0, comm, True)
        torch.cuda.synchronize(dev)
        node_s.append(time.perf_counter() - t0)
        rec_bytes.append(lw.stats()["node_record_bytes"] - rb0)
        coll_us.append(lw.node_collective_us())
        got = out.cpu().numpy().astype(np.float64)
        ref = np.full((S, 8), np.nan)
        s0 = 0
        for i, w in enumerate(WIDTHS):
            union = np.concatenate([mirrors[q][i] for q in range(world)])  # [sum_n, w]
            st = window_stats_reference(union.T)
            st[:, 6] = np.nan  # no node-wide newest sample
            ref[s0:s0 + w] = st
            s0 += w
        # min, max, count: exact; the percentiles interpolate two exact order statistics
        # in fp64 and round to float32 - a tie (the midpoint of two neighbouring float32
        # samples) may round either way against numpy's fp64 lerp: within 1 float32 ulp
        order = [0, 1, 7]
        if not np.array_equal(np.float32(got[:, order]), np.float32(ref[:, order]), equal_nan=True):
            bad = np.argwhere(np.float32(got[:, order]) != np.float32(ref[:, order]))
            errors.append(f"rank {rank} step {step}: min / max / count differ at {bad[:4].tolist()}")
        g32, r32 = np.float32(got[:, 3:6]), np.float32(ref[:, 3:6])
        ulp = np.spacing(np.abs(r32))
        fin = np.isfinite(r32)
        if not (np.array_equal(np.isnan(g32), np.isnan(r32)) and np.all(np.abs(g32[fin] - r32[fin]) <= ulp[fin])):
            bad = np.argwhere(~(np.abs(g32 - r32) <= ulp) & fin)
            errors.append(f"rank {rank} step {step}: percentiles differ by > 1 ulp at {bad[:4].tolist()}: "
                          f"{g32[tuple(bad[0])] if len(bad) else ''} vs {r32[tuple(bad[0])] if len(bad) else ''}")
        if not np.allclose(got[:, 2], ref[:, 2], rtol=1e-5, equal_nan=True):
            errors.append(f"rank {rank} step {step}: mean differs")
        if not np.isnan(got[:, 6]).all():
            errors.append(f"rank {rank} step {step}: last is not NaN")
        checks += 1
    st = lw.stats()
    if st["rows_lost"]:
        errors.append(f"rank {rank}: {st['rows_lost']} rows lost (plan exceeds the host ring)")
    errs = agg.all_gather_object(errors)
    all_errors = [e for es in errs for e in es]
    if rank == 0:
        from rocmdash.parallel.node_window import NodeWindowStats

        names = NodeWindowStats.COLLECTIVE_STEPS
        steady = node_s[-args.steady // 2:] if args.steady >= 4 else node_s

        def p50(i):
            v = [c[i] for c in coll_us if c and c[i] == c[i]]
            return round(statistics.median(v), 2) if v else None

        print(json.dumps({
            "ok": not all_errors,
            "world": world,
            "oversubscribed": oversubscribed(),
            "window": W,
            "series": S,
            "node_refreshes": checks,
            "node_refresh_ms_p50": round(statistics.median(node_s) * 1e3, 3) if node_s else None,
            "steady_node_refresh_ms_p50": round(statistics.median(steady) * 1e3, 3) if steady else None,
            "brackets": not args.no_brackets,
            "node_fused_passb": bool(args.node_fused),
            "collective_us_p50": {n: p50(i) for i, n in enumerate(names)} if coll_us and coll_us[0] else None,
            "stats": st,
            # the records shrink to the node's kept keys (lw_node_cap_next) after the first hit
            "record_bytes_first_last": [next((b for b in rec_bytes if b), 0), rec_bytes[-1] if rec_bytes else 0],
            # node refreshes each series resolved from the node's brackets
            "node_bracket_hits": [x[1] for x in lw.bracket_stats(1)],
            "errors": all_errors[:10],
        }), flush=True)
    if agg.native is not None:
        agg.native.close()
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()
    return 0 if not all_errors else 1


if __name__ == "__main__":
    raise SystemExit(main())
