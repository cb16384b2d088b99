#!/usr/bin/env python3
"""Table of a bench_long_window.py A/B log: per (W, data, set) the median over rounds of
the per-refresh p50 µs, its chunk rows, and the window bandwidth (W x series x 4 B per
refresh-time; one streaming pass of the window at that rate)."""

import json
import statistics
import sys
from collections import defaultdict


def main(path: str) -> int:
    rows = defaultdict(list)
    meta = {}
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "launch" not in d:
            continue
        key = (d["W"], d["data"], d["launch"])
        rows[key].append(d["p50_us"])
        meta[key] = d
    last = None
    for (W, data, launch), v in sorted(rows.items(), key=lambda kv: (kv[0][0], kv[0][1], statistics.median(kv[1]))):
        if (W, data) != last:
            print(f"W={W} data={data}")
            last = (W, data)
        m = statistics.median(v)
        d = meta[(W, data, launch)]
        print(f"  {launch:22s} chunk {d['chunk_rows']:6d}  p50 {m:9.1f} us  rounds {[round(x, 1) for x in v]}  "
              f"window {d['window_bytes'] / (m * 1e-6) / 1e12:5.2f} TB/s per refresh")
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1]))
