#!/usr/bin/env python3
"""Multi-rank check of the native N > 1 gather on real GPUs (one rank per process).

Run under torchrun; on a box with fewer GPUs than ranks set ROCMDASH_OVERSUBSCRIBE=1
(every rank drives GPU ``rank % GPUs`` and RCCL connects the ranks over sockets - see
rocmdash.parallel.node.oversubscribed):

    ROCMDASH_OVERSUBSCRIBE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \\
        --master-addr 127.0.0.1 --master-port 29541 tools/multirank_check.py --refreshes 40

Every rank builds the service's pipeline (health / XCD / control rows, HIP-event timing)
on synthetic sources seeded per rank (distinct data on every rank), so that:
  * the pipeline must be on the native path (one RCCL communicator per process, gloo
    control plane) with its start-up gathers validated bit for bit;
  * rank 0's node tensor, refresh after refresh, equals every rank's own statistics in
    rank order (checked against an all_gather_object of the ranks' own blocks);
  * every rank sees every rank's stop vote; the per-rank footprint rows arrive;
  * the node-window statistics gather goes through the same communicator and matches
    the fp64 reference of the union of the ranks' windows;
  * HIP-event stage times of the native ncclAllGather and publish kernel are recorded.
Rank 0 prints one JSON line; exit code 0 only if every check passed on every rank.
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


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--refreshes", type=int, default=40)
    ap.add_argument("--window", type=int, default=512)
    ap.add_argument("--node-window", type=int, default=1)
    ap.add_argument("--node-window-reps", type=int, default=0,
                    help="then time this many node-window refreshes (the all-gather of every rank's sorted window "
                    "+ the selection; VERDICT r05 item 7: default vs the supervisor's lean RCCL environment)")
    args = ap.parse_args(argv)

    from rocmdash.runtime import native

    native.load()
    import numpy as np
    import torch

    from rocmdash.config import SamplerConfig
    from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ, oversubscribed
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.footprint import Footprint, decode_control
    from rocmdash.runtime.pipeline import NodePipeline

    env = dist_env_from_environ(prefer_gpu=True, timeout_s=120)
    rank, world = env.rank, env.world_size
    errors = []

    def check(cond, msg):
        if not cond:
            errors.append(f"rank {rank}: {msg}")

    fp = Footprint(env.device)
    fp.mark("start")
    cfg = SamplerConfig(window=args.window, ring_capacity=max(4 * args.window, 4096))
    agent = GpuAgent(env.device.index, source="synthetic", counters="synthetic", cfg=cfg, use_gpu=True,
                     seed=1000 + 17 * rank)
    agent.prefill(args.window + 8)
    fp.mark("agent")
    agg = NodeAggregator()
    check(agg.backend == "gloo", f"control plane is {agg.backend}, not gloo")
    pipe = NodePipeline(agent, agg, health=True, device_timing=True)
    pipe.footprint = fp
    fp.mark("pipeline")
    rep = pipe.gather_report()
    check(rep["status"] == "native", f"gather status {rep}")
    S = len(agent.series)
    stage = {}
    t0 = time.perf_counter()
    for i in range(args.refreshes):
        agent.sample()
        pipe.stop_vote = 1.0 if (i == args.refreshes - 1 and rank == world - 1) else 0.0
        snap = pipe.latest_snapshot()
        votes = pipe.stop_votes()
        want_votes = [0.0] * world if i < args.refreshes - 1 else [0.0] * (world - 1) + [1.0]
        check(votes is not None and votes.tolist() == want_votes, f"refresh {i}: votes {votes}")
        own = agent.refresh().clone()  # the same window again: this rank's statistics
        torch.cuda.synchronize(env.device)
        blocks = agg.all_gather_object(own.cpu().numpy())
        if rank == 0:
            check(snap is not None and snap.window.shape == (world, S, 8), "snapshot shape")
            if snap is not None:
                a = np.ascontiguousarray(snap.window, dtype=np.float32)
                b = np.stack(blocks).astype(np.float32)
                check(np.array_equal(a.view(np.int32), b.view(np.int32)), f"refresh {i}: node tensor != rank blocks")
                ctl = pipe.last_control
                check(ctl is not None and ctl.shape[0] == world, "control rows")
                for r in range(world):
                    d = decode_control(ctl[r])
                    check(d["native_gather"] == 1.0, f"refresh {i}: rank {r} native_gather {d['native_gather']}")
                    check(d["rss_bytes"] and d["rss_bytes"] > 0 and d["cpu_seconds"] is not None, f"footprint {d}")
            for k, v in pipe.stage_seconds().items():
                stage.setdefault(k, []).append(v * 1e6)
        else:
            check(snap is None, "non-root snapshot")
    dt = time.perf_counter() - t0
    rep = pipe.gather_report()
    check(rep["status"] == "native" and rep["validated"] == rep["validate_target"] > 0, f"after the run: {rep}")

    nw = None
    if args.node_window:
        from rocmdash.parallel.node_window import NodeWindowStats, node_window_reference

        nws = NodeWindowStats(agent, agg)
        agent.refresh()
        got = nws.refresh()
        blk = agent.export_window().cpu().numpy()
        blocks = agg.all_gather_object(blk)
        if rank == 0:
            ref = node_window_reference(np.stack(blocks))
            ok = np.allclose(got.cpu().numpy(), ref, rtol=1e-5, atol=1e-3, equal_nan=True)
            check(ok, "node-window statistics over the native gather differ from the fp64 reference")
            nw = bool(ok)
        nw_ms = []
        for _ in range(args.node_window_reps):
            agg.barrier()
            t1 = time.perf_counter()
            got = nws.refresh()
            if got is not None:
                got.cpu()
            torch.cuda.synchronize(env.device)
            nw_ms.append((time.perf_counter() - t1) * 1e3)
        nw_ms.sort()
    # RCCL's own view of every rank's communicator and the transports it logged per peer
    rv = agg.all_gather_object({k: rep.get(k) for k in ("rccl_nranks", "rccl_rank", "rccl_device")}
                               | {"kinds": (rep.get("transport_detail") or {}).get("kinds")})
    for r, v in enumerate(rv):
        check(v["rccl_nranks"] == world and v["rccl_rank"] == r, f"RCCL's view of rank {r}: {v}")
    agg.barrier()
    errs = agg.all_gather_object(errors)
    all_errors = [e for es in errs for e in es]
    if rank == 0:
        out = {
            "ok": not all_errors,
            "world": world,
            "gpus_visible": torch.cuda.device_count(),
            "oversubscribed": oversubscribed(),
            "transport": rep["transport"],
            "gather_validated": rep["validated"],
            "refreshes": args.refreshes,
            "refresh_ms_mean": round(dt / args.refreshes * 1e3, 3),
            "stage_us_p50": {k: round(statistics.median(v), 2) for k, v in stage.items()},
            "node_window_ok": nw,
            "node_window_ms": None if not args.node_window or not args.node_window_reps else {
                "p50": round(statistics.median(nw_ms), 3), "p90": round(nw_ms[int(0.9 * len(nw_ms))], 3),
                "n": len(nw_ms), "bytes_per_rank": int(S * (args.window + 1) * 4),
                "env": {k: os.environ.get(k) for k in ("NCCL_MAX_NCHANNELS", "NCCL_BUFFSIZE", "GPU_MAX_HW_QUEUES")}},
            "rccl_views": rv,
            "footprint_rank0": {k: {kk: vv for kk, vv in v.items() if vv is not None} for k, v in fp.stages.items()},
            "errors": all_errors[:20],
        }
        print(json.dumps(out), flush=True)
    pipe.close()
    agent.close()
    import torch.distributed as dist

    dist.destroy_process_group()
    return 0 if not all_errors else 1


if __name__ == "__main__":
    raise SystemExit(main())
