"""Long-window statistics micro-benchmark (csrc/long_window.hip): one refresh with
``--new-rows`` new rows per ring (default 1; the service at 100 Hz / 1 Hz: 100) over an HBM-resident window of W samples per series (8 + 4 series),
graph vs direct launches, chunk size sized from W vs fixed 4096-row chunks, on two
data shapes: "normal" (continuous, N(50, 10) / N(500, 100): at 2^16+ samples the far tails
cross zero, so the sign bit varies), "positive" (|N| + 1, never negative) and "telemetry"
(integer-valued readings in a narrow band, as temperatures / power / activity are);
effective bandwidth = 4 passes x W x series x 4 B / time (the first version's 4 full
streams; the adaptive digits stream the window 1-3 times, by how many key bits vary),
window_GBps = W x 12 x 4 B / time.

    python tools/bench_long_window.py [--windows 65536,1048576,4194304,16777216] [--out x.json]
"""

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", default="65536,1048576,4194304,16777216")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="normal,positive,telemetry")
    ap.add_argument("--chunks", default="", help="extra direct-launch sets with these chunk_rows (A/B)")
    ap.add_argument("--rounds", type=int, default=1, help="time every set this many times, alternating")
    ap.add_argument("--wave-private-ab", action="store_true", help="add a set with pass 0's shared LDS histogram")
    ap.add_argument("--compact-ab", action="store_true", help="add a set without candidate compaction")
    ap.add_argument("--half-wave-ab", action="store_true", help="add a set with pass 0's half-wave LDS copies")
    ap.add_argument("--old-ab", action="store_true", help="add the round-3 configuration")
    ap.add_argument("--prefetch-ab", action="store_true", help="add a set without the next-rows prefetch")
    ap.add_argument("--brackets-ab", action="store_true", help="add a set with the radix chain alone (no bracket mode)")
    ap.add_argument("--incremental-ab", action="store_true",
                    help="add a set with bracket mode streaming the whole window every refresh (round 4)")
    ap.add_argument("--plan-rounds-ab", default="", help="extra direct sets planned with these rounds (A/B)")
    ap.add_argument("--brk-target-ab", default="", help="extra direct sets with these bracket targets (A/B)")
    ap.add_argument("--fused-ab", action="store_true",
                    help="add a set whose incremental pass B is always its own kernel (not fused into scan B)")
    ap.add_argument("--layout", default="8+4",
                    help="series per ring, '+'-separated (8+4: the service's two rings; 8 / 4 / 12 / 4+4+4 "
                         "isolate how the rings' workgroups share the chip)")
    ap.add_argument("--new-rows", type=int, default=1,
                    help="rows entering per refresh (the service at 100 Hz sampling, 1 Hz refresh: 100)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch

    from rocmdash.runtime import native

    nat = native.load()
    nat.set_pinned_host_rings(True)
    rows = []
    shapes = args.shapes.split(",")
    for W in [int(w) for w in args.windows.split(",")]:
        for shape in shapes:
            cap = min(W, 1 << 20)
            widths = [int(x) for x in args.layout.split("+")]
            nser = sum(widths)
            rings = [nat.SeriesRing(wd, cap) for wd in widths]
            # graph launch with the chunk size sized from W (default) vs direct launches vs
            # the fixed 4096-row chunks of the first version
            sets = {"graph": nat.LongWindowSet(W, 0, True), "direct": nat.LongWindowSet(W, 0, False),  # direct: default
                    "graph_chunk4096": nat.LongWindowSet(W, 0, True, 4096)}
            for c in [int(x) for x in args.chunks.split(",") if x]:
                if c <= W:
                    sets[f"direct_chunk{c}"] = nat.LongWindowSet(W, 0, False, c)
            if args.wave_private_ab:  # pass 0 with one shared LDS histogram (the pre-r4 form)
                sets["direct_shared_lds"] = nat.LongWindowSet(W, 0, False)
                sets["direct_shared_lds"].wave_private = False
            if args.half_wave_ab:  # pass 0: an LDS histogram copy per half wave
                sets["direct_halfwave"] = nat.LongWindowSet(W, 0, False)
                sets["direct_halfwave"].wave_private_level = 2
            if args.compact_ab:  # pass 3 streams the window again (no candidate compaction)
                sets["direct_no_compact"] = nat.LongWindowSet(W, 0, False)
                sets["direct_no_compact"].compact = False
            if args.prefetch_ab:  # the other prefetch modes
                for mode in (0, 1, 2):
                    sets[f"direct_prefetch{mode}"] = nat.LongWindowSet(W, 0, False)
                    sets[f"direct_prefetch{mode}"].prefetch = mode
            if args.brackets_ab:  # every refresh through the radix passes 0-3
                sets["direct_radix"] = nat.LongWindowSet(W, 0, False)
                sets["direct_radix"].brackets = False
            if args.incremental_ab:  # pass B over every chunk, the radix chain enqueued behind it
                sets["direct_full_passb"] = nat.LongWindowSet(W, 0, False)
                sets["direct_full_passb"].incremental = False
            for n in [int(x) for x in args.plan_rounds_ab.split(",") if x]:
                sets[f"direct_rounds{n}"] = nat.LongWindowSet(W, 0, False)
                sets[f"direct_rounds{n}"].plan_rounds = n
                if args.brackets_ab:  # the full radix chain with that plan (a miss's cost)
                    sets[f"direct_rounds{n}_radix"] = nat.LongWindowSet(W, 0, False)
                    sets[f"direct_rounds{n}_radix"].plan_rounds = n
                    sets[f"direct_rounds{n}_radix"].brackets = False
            if args.fused_ab:
                sets["direct_unfused"] = nat.LongWindowSet(W, 0, False)
                sets["direct_unfused"].fused_passb = False
            for n in [int(x) for x in args.brk_target_ab.split(",") if x]:
                sets[f"direct_target{n}"] = nat.LongWindowSet(W, 0, False)
                sets[f"direct_target{n}"].brk_target = n
            if args.old_ab:  # the round-3 configuration: 4096-row chunks, shared LDS, no compaction
                sets["direct_r3"] = nat.LongWindowSet(W, 0, False, 4096)
                sets["direct_r3"].wave_private = False
                sets["direct_r3"].compact = False
                sets["direct_r3"].prefetch = 0
            for s in sets.values():
                for ring in rings:
                    s.add_ring(ring)
            outs = {k: torch.empty((nser, 8), device="cuda") for k in sets}
            stream = torch.cuda.current_stream().cuda_stream
            rng = np.random.default_rng(0)
            t = 0
            if shape == "telemetry":  # integer readings in a narrow band (temps, W, %)
                gen = [lambda n: rng.integers(40, 56, (cap, n)), lambda n: rng.integers(700, 760, (cap, n))]
            elif shape == "positive":  # continuous, never negative (bandwidth, utilisation)
                gen = [lambda n: np.abs(rng.normal(50, 10, (cap, n))) + 1,
                       lambda n: np.abs(rng.normal(500, 100, (cap, n))) + 1]
            else:  # continuous with mixed signs in the far tails (the sign bit varies)
                gen = [lambda n: rng.normal(50, 10, (cap, n)), lambda n: rng.normal(500, 100, (cap, n))]
            # ring 0 holds the first kind (temperatures, activity), later rings the second (power)
            blocks = [gen[min(i, 1)](wd).astype(np.float32) for i, wd in enumerate(widths)]
            while t < W:  # fill the window through the host ring, one ring-full at a time
                ts = np.arange(t, t + cap, dtype=np.uint64)
                for ring, blk in zip(rings, blocks):
                    ring.push_many(blk, ts)
                t += cap
                for k, s in sets.items():
                    s.refresh(outs[k].data_ptr(), stream)
            torch.cuda.synchronize()
            for name, s in [kv for _ in range(args.rounds) for kv in sets.items()]:
                out = outs[name]
                st0 = s.stats()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
                for i in range(args.iters + 5):
                    k = args.new_rows
                    o = (t * 7919) % (cap - k) if cap > k else 0  # a different slice of the block each time
                    for ring, blk in zip(rings, blocks):
                        ring.push_many(blk[o:o + k], np.arange(t, t + k, dtype=np.uint64))
                    t += k
                    if i >= 5:
                        ev[i - 5][0].record()
                    s.refresh(out.data_ptr(), stream)
                    if i >= 5:
                        ev[i - 5][1].record()
                torch.cuda.synchronize()
                us = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
                p50 = statistics.median(us)
                st1 = s.stats()
                n = args.iters + 5
                per = {k: round((st1.get(k, 0) - st0.get(k, 0)) / n, 2)
                       for k in ("passb_chunks", "chain_refreshes", "kernel_launches", "fused_refreshes",
                                 "single_kernel_refreshes")}
                per.update({k.replace("_ns", "_us"): round((st1.get(k, 0) - st0.get(k, 0)) / n / 1e3, 2)
                            for k in ("host_stage_ns", "host_enqueue_ns", "host_wait_ns")})
                gbs = 4 * W * nser * 4 / (p50 * 1e-6) / 1e9
                rows.append({"W": W, "data": shape, "layout": args.layout, "new_rows": args.new_rows, "launch": name,
                             "chunk_rows": s.chunk_rows,
                             "p50_us": round(p50, 1), "min_us": round(us[0], 1),
                             "effective_GBps": round(gbs, 1), "window_GBps": round(gbs / 4, 1),
                             "window_bytes": W * nser * 4, "incremental": bool(getattr(s, "incremental", False)),
                             "per_refresh": per})
                print(json.dumps(rows[-1]), flush=True)
            # one more refresh of every set over the same rows: every order statistic agrees
            # bit for bit (the mean is summed per chunk, so only to rounding)
            for k, s in sets.items():
                s.refresh(outs[k].data_ptr(), stream)
            torch.cuda.synchronize()
            keep = [0, 1, 3, 4, 5, 6, 7]
            ref = outs["graph_chunk4096"]
            agree = all(torch.equal(o[:, keep].nan_to_num(-7.0), ref[:, keep].nan_to_num(-7.0))
                        and torch.allclose(o[:, 2], ref[:, 2], rtol=1e-6) for o in outs.values())
            print(json.dumps({"W": W, "data": shape, "variants_agree": agree}), flush=True)
            if not agree:
                raise SystemExit(f"long-window variants disagree at W={W} data={shape}")
            hits = {k: [x[1] for x in s.bracket_stats()] for k, s in sets.items() if s.brackets}
            print(json.dumps({"W": W, "data": shape, "bracket_hits_per_series": hits.get("direct")}), flush=True)
            del sets
            torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
