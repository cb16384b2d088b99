#!/usr/bin/env python3
"""Micro-benchmark of the window-stats refresh on one GPU (device time per refresh).

For each window W and series count S, a pinned host ring feeds a DeviceWindowSet;
every timed refresh first pushes k new rows, then enqueues the delta copy + the
stats launch; HIP events bracket the refresh on the stream. k <= 256 takes the
incremental path (resident sorted window), k > 256 the full bitonic sort; the
stateless ``window_stats_raw`` full sort is timed too.

    python tools/bench_kernel.py [--iters 200] [--out file.json]
Profile: rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python3 tools/bench_kernel.py
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--windows", type=int, nargs="+", default=[1024, 4096, 16384])
    ap.add_argument("--series", type=int, nargs="+", default=[12, 64])
    ap.add_argument("--ks", type=int, nargs="+", default=[1, 10, 100, 300])
    ap.add_argument("--rings", type=int, nargs="+", default=None,
                    help="ring widths of ONE set instead of --series (the headline's launch: --rings 11 5 = the amd-smi "
                    "ring + the device-counter ring, 16 series in a max(cols) x rings grid)")
    ap.add_argument("--signal", type=int, default=0, choices=[0, 1, 2],
                    help="completion signal: 0 none (device outputs, the N > 1 shape), 1 last-workgroup flag, "
                    "2 tagged host outputs (the N = 1 host-out refresh; waited for with wait_done)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)

    import numpy as np

    from rocmdash.runtime import native

    nat = native.load()
    import torch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nat.set_pinned_host_rings(True)
    stream = torch.cuda.current_stream(dev)
    rows_out = []
    rng = np.random.default_rng(0)
    for W in args.windows:
        for widths in ([tuple(args.rings)] if args.rings else [(S,) for S in args.series]):
            S = sum(widths)
            rings = [nat.SeriesRing(w, max(8 * W, 16384)) for w in widths]
            offs = np.cumsum((0,) + widths)[:-1]
            dws = nat.DeviceWindowSet(W, 0)
            for ring in rings:
                dws.add_ring(ring)

            def push(rows, stamps):
                for ring, o, w in zip(rings, offs, widths):
                    ring.push_many(np.ascontiguousarray(rows[:, o:o + w]), stamps)
            out = (torch.empty((S, 8), pin_memory=True) if args.signal == 2 else torch.empty((S, 8), device=dev))
            block = rng.integers(0, 400, size=(4 * W, S)).astype(np.float32)
            ts = np.arange(4 * W, dtype=np.uint64)
            push(block[:W], ts[:W])
            dws.refresh(out.data_ptr(), stream.cuda_stream, signal=args.signal)
            torch.cuda.synchronize()
            pos = W
            for k in args.ks:
                times = []
                for _ in range(args.iters):
                    if pos + k > len(block):
                        pos = W
                    push(block[pos : pos + k], ts[pos : pos + k])
                    pos += k
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    seq = dws.refresh(out.data_ptr(), stream.cuda_stream, signal=args.signal)
                    e1.record(stream)
                    e1.synchronize()
                    if args.signal == 2 and not dws.wait_done(seq, 1.0):
                        raise RuntimeError("tagged outputs never arrived")
                    times.append(e0.elapsed_time(e1) * 1e3)
                times = sorted(times[10:])
                row = {
                    "W": W, "series": S, "rings": list(widths), "k_new": k, "signal": args.signal, "path": "incremental" if k <= 256 else "full",
                    "p50_us": round(statistics.median(times), 2), "min_us": round(times[0], 2),
                }
                rows_out.append(row)
                print(json.dumps(row), flush=True)
            # stateless full sort over a device tensor (no copies)
            from rocmdash.ops.window_stats import window_stats

            x = torch.randint(0, 400, (S, W), device=dev).float()
            window_stats(x)
            times = []
            for _ in range(args.iters):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                window_stats(x)
                e1.record(stream)
                e1.synchronize()
                times.append(e0.elapsed_time(e1) * 1e3)
            times = sorted(times[10:])
            row = {"W": W, "series": S, "k_new": None, "path": "stateless-full (incl. transpose copy)",
                   "p50_us": round(statistics.median(times), 2), "min_us": round(times[0], 2)}
            rows_out.append(row)
            print(json.dumps(row), flush=True)
            del dws
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows_out, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
