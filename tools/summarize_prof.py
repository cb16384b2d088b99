#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace / PMC counter collection) into a small
JSON for profiles/: per kernel the dispatch count, duration percentiles and the mean
of every collected counter per dispatch.

    python tools/summarize_prof.py gpurun_out/prof_kernel/run_kernel_trace.csv [--pmc file] --out profiles/x.json
"""

from __future__ import annotations

import argparse
import collections
import csv
import json
import statistics


def short(name: str) -> str:
    name = name.replace("rocmdash::(anonymous namespace)::", "")
    return name if len(name) < 120 else name[:117] + "..."


def kernel_trace(path: str) -> dict:
    durs = collections.defaultdict(list)
    meta = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
            meta[k] = {x: r.get(x) for x in ("Workgroup_Size_X", "Grid_Size_X", "LDS_Block_Size", "VGPR_Count", "SGPR_Count", "Scratch_Size")}
    out = {}
    for k, d in durs.items():
        d.sort()
        out[k] = {
            "dispatches": len(d),
            "p50_us": round(statistics.median(d), 2),
            "p10_us": round(d[len(d) // 10], 2),
            "p90_us": round(d[min(len(d) - 1, 9 * len(d) // 10)], 2),
            "total_us": round(sum(d), 1),
            **meta[k],
        }
    return out


def pmc(path: str) -> dict:
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: {"dispatches": len(disp[k]), **{c: round(v / len(disp[k]), 1) for c, v in cs.items()}} for k, cs in sums.items()}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="?")
    ap.add_argument("--pmc", default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    args = ap.parse_args(argv)
    res = {"note": args.note}
    if args.trace:
        res["kernels"] = kernel_trace(args.trace)
    if args.pmc:
        res["pmc_per_dispatch"] = pmc(args.pmc)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1)[:3000])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
