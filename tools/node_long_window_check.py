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

``--full-cap``: one column (series 10) is a grid interleaved over the
ranks - rank r's row t holds world x bitrev(t mod W) + r, so the node window's values are
exactly 0 .. world W - 1 and any value interval holds the same number of every rank's
samples. After the plan the node state is reset (``reset_node``: records at kNodeCap),
one chain refresh sets brackets, and the check then sets that series' three node brackets
(``set_node_brackets``) so that EVERY rank keeps exactly kNodeCap = 1024 keys in each:
scan B selects among world x 1024 keys - 8192 at 8 ranks, its LDS bound (kBrkCap).
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


GRID_SERIES = 10  # --full-cap: ring 1 (width 4), column 2


def bitrev(x, bits: int):
    import numpy as np

    x = np.asarray(x, dtype=np.uint64)
    out = np.zeros_like(x)
    for b in range(bits):
        out |= ((x >> np.uint64(b)) & np.uint64(1)) << np.uint64(bits - 1 - b)
    return out


def rows_for(rank: int, step: int, k: int, t0: int, grid=None):
    """``grid`` = (world, window): series GRID_SERIES is the interleaved grid column."""
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
        if grid is not None and w == 4:
            world, W = grid
            t = np.arange(t0, t0 + k, dtype=np.uint64) % np.uint64(W)
            x[:, GRID_SERIES - WIDTHS[0]] = (bitrev(t, W.bit_length() - 1) * np.uint64(world) +
                                             np.uint64(rank)).astype(np.float32)
        out.append(x)
    return out


def fkey(v: float) -> int:
    """csrc/long_window.hip fkey: the order-preserving uint32 key of a float32."""
    import numpy as np

    u = int(np.array([v], np.float32).view(np.uint32)[0])
    return (~u) & 0xFFFFFFFF if u & 0x80000000 else u | 0x80000000


def full_cap_brackets(world: int, W: int, pct, per_rank: int = 1024):
    """Three node brackets around the percentile positions of the grid column holding
    exactly ``per_rank`` keys of every rank strictly inside (bounds excluded)."""
    import math

    nv = world * W
    lo, hi = [], []
    for p in pct:
        c = int(math.floor(p / 100.0 * (nv - 1)))  # the sorted union is 0 .. nv - 1: value = position
        v_lo = c - world * per_rank // 2 - 1
        v_hi = v_lo + world * per_rank + 1
        assert v_lo >= 0 and v_hi < nv and v_lo < c and c + 1 < v_hi
        lo.append(fkey(float(v_lo)))
        hi.append(fkey(float(v_hi)))
    return lo, hi


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--window", type=int, default=1 << 20)
    ap.add_argument("--capacity", type=int, default=1 << 17)
    ap.add_argument("--no-brackets", action="store_true", help="radix chain on every node refresh")
    ap.add_argument("--steady", type=int, default=24, help="node refreshes of 100-row pushes at the end (bracket hits)")
    ap.add_argument("--full-cap", action="store_true",
                    help="end with a node bracket refresh in which every rank keeps kNodeCap keys of one bracket")
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
    if args.full_cap:
        plan += [("reset", 0), ("node", 100), ("fullcap", 100)] + [("node", 100)] * 4
    grid = (world, W) if args.full_cap else None
    full = None
    coll_us = []
    checks = 0
    t = 0
    node_s = []
    rec_bytes = []  # this rank's all-gathered bracket records per node refresh (0: none)
    for step, (kind, k) in enumerate(plan):
        if kind == "reset":  # every rank: the node state a new membership epoch starts from
            lw.reset_node()
            continue
        for q in range(world):
            xs = rows_for(q, step, k, t, grid)
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
        if kind == "fullcap":
            blo, bhi = full_cap_brackets(world, W, (50.0, 90.0, 99.0))
            lw.set_node_brackets(GRID_SERIES, blo, bhi)
            full = {"node_cap": lw.node_cap, "hits_before": lw.bracket_stats(1)[GRID_SERIES][1]}
        t0 = time.perf_counter()
        lw.refresh_node(out.data_ptr(), stream, 50.0, 90.0, 99.0, comm, True)
        torch.cuda.synchronize(dev)
        node_s.append(time.perf_counter() - t0)
        rec_bytes.append(lw.stats()["node_record_bytes"] - rb0)
        if kind == "fullcap":
            full.update(maxmid=lw.node_last_maxmid, record_bytes=rec_bytes[-1],
                        hit=lw.bracket_stats(1)[GRID_SERIES][1] > full.pop("hits_before"),
                        union_keys_per_bracket=world * 1024)
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
            "collective_us_p50": {n: p50(i) for i, n in enumerate(names)} if coll_us and coll_us[0] else None,
            "stats": st,
            # the records shrink to the node's kept keys (lw_node_cap_next) after the first hit
            "record_bytes_first_last": [next((b for b in rec_bytes if b), 0), rec_bytes[-1] if rec_bytes else 0],
            # node refreshes each series resolved from the node's brackets
            "node_bracket_hits": [x[1] for x in lw.bracket_stats(1)],
            "full_cap": full,
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
