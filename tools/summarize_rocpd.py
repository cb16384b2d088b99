#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd database (ROCm 7.2's default output):
name, calls, total / mean / p50 / min / max duration (µs), grid and workgroup.

    python tools/summarize_rocpd.py gpurun_out/.../run_results.db [--csv out.csv]
"""
import argparse
import csv
import sqlite3
import statistics
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    args = ap.parse_args(argv)
    c = sqlite3.connect(args.db)
    rows = c.execute("select name, duration, grid_x, grid_y, workgroup_x from kernels").fetchall()
    by = {}
    for name, dur, gx, gy, wx in rows:
        by.setdefault(name, {"d": [], "shape": (gx, gy, wx)})["d"].append(dur / 1e3)
    out = []
    for name, v in by.items():
        d = sorted(v["d"])
        out.append({"kernel": name[:120], "calls": len(d), "total_us": round(sum(d), 1), "mean_us": round(sum(d) / len(d), 2),
                    "p50_us": round(statistics.median(d), 2), "min_us": round(d[0], 2), "max_us": round(d[-1], 2),
                    "grid_xy_wg": "x".join(map(str, v["shape"]))})
    out.sort(key=lambda r: -r["total_us"])
    w = csv.DictWriter(sys.stdout, fieldnames=list(out[0]))
    w.writeheader()
    w.writerows(out)
    if args.csv:
        with open(args.csv, "w", newline="") as f:
            w2 = csv.DictWriter(f, fieldnames=list(out[0]))
            w2.writeheader()
            w2.writerows(out)


if __name__ == "__main__":
    main()
