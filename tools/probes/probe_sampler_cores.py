"""Per-core cost of one amd-smi (raw SMU table) and one device-counter sample.

The sampler's read time is bimodal across runs on the MI355X box (~50/72 us vs
~110/139 us for the SMU / counter reads, profiles/r01/handoff_*.json), independent
of spin / NUMA pinning. This pins the sampler worker threads to one core at a time
(a spread over the allowed, GPU-local CPUs) and reports the median read time per
core, to see whether the cost is a property of the core the thread runs on.

    python tools/probes/probe_sampler_cores.py [--per-core 200] [--stride 8]
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
    ap.add_argument("--per-core", type=int, default=200)
    ap.add_argument("--stride", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from rocmdash.runtime import native

    nat = native.load()
    native.enable_counters(only_device=0)
    from rocmdash.runtime.agent import numa_local_cpus

    bdf = int(nat.hip_device_bdf(0))
    smi = nat.make_smi_source(bdf, 0)
    srcs = [("smi", smi)]
    if native.counters_ready():
        srcs.append(("ctr", nat.make_counter_source(bdf, 0)))
    allowed = sorted(os.sched_getaffinity(0))
    local = numa_local_cpus(bdf) or allowed
    cand = local[:: max(1, args.stride)]
    rows = []

    def run(cpus):
        res = {}
        for name, src in srcs:
            ring = nat.SeriesRing(src.width, 1024)
            s = nat.Sampler(src, ring, 10.0)
            s.set_spin_us(200.0)
            if cpus:
                s.set_affinity(cpus)
            lat = []
            for _ in range(args.per_core):
                t0 = time.perf_counter()
                s.request()
                s.wait()
                lat.append((time.perf_counter() - t0) * 1e6)
            st = s.stats()
            res[name] = {"read_p50_us": round(st["p50_us"], 1), "handoff_p50_us": round(statistics.median(lat), 1)}
            del s
        return res

    rows.append({"cpu": "unpinned", **run([])})
    print(json.dumps(rows[-1]), flush=True)
    for c in cand:
        rows.append({"cpu": c, **run([c])})
        print(json.dumps(rows[-1]), flush=True)
    rows.append({"cpu": "unpinned-end", **run([])})
    print(json.dumps(rows[-1]), flush=True)
    info = {"allowed_cpus": len(allowed), "local_cpus": len(local), "rows": rows}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(info, f, indent=1)


if __name__ == "__main__":
    main()
