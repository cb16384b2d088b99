#!/usr/bin/env python3
"""Per-pass kernel times of a bench_long_window.py trace, by timed block: the bench runs
every set's refreshes back to back (5 warm-up + --iters timed), so consecutive refreshes
(a refresh starts at lw_pass_brk, or at lw_pass<0> without bracket mode) with the same launch shape form a block; prints each
block's median µs per kernel and its window bandwidth per streaming pass."""

import csv
import statistics
import sys
from collections import OrderedDict


def main(path: str, min_refreshes: int = 15) -> int:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    refreshes = []
    cur = None
    last = None
    for r in rows:
        name = r["Kernel_Name"]
        if "lw_" not in name:
            continue
        short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].replace("rocmdash::", "")
        # a refresh starts at pass B (bracket mode) or at pass 0 not preceded by scan B
        starts = short.startswith("lw_pass_brk") or (
            (short.startswith("lw_pass<0>") or short.startswith("lw_pass<0,")) and last != "lw_scan_brk")
        last = short
        if starts:
            cur = OrderedDict()
            cur["_grid"] = r["Grid_Size_X"]
            refreshes.append(cur)
        if cur is None:
            continue
        cur[short] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    blocks = []
    for ref in refreshes:
        key = (ref["_grid"], tuple(k for k in ref if k != "_grid"))
        if blocks and blocks[-1][0] == key:
            blocks[-1][1].append(ref)
        else:
            blocks.append((key, [ref]))
    for (grid, names), refs in blocks:
        if len(refs) < min_refreshes:
            continue
        med = {k: statistics.median(r[k] for r in refs) for k in names}
        tot = sum(med.values())
        print(f"block of {len(refs)} refreshes, pass grid {grid}: total {tot:.1f} us  " +
              "  ".join(f"{k}={v:.1f}" for k, v in med.items()))
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15))
