#!/bin/bash
# Same-box A/B of the long-window kernel: the tree at OLD (a git worktree at ./ab_old,
# built in place, with this tree's tools/bench_long_window.py copied in) vs this tree,
# 3 alternating rounds. Usage (via gpurun): bash tools/ab_long_window.sh [out_dir]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/ab_lw}; mkdir -p "$O"
python3 -m rocmdash._build --check || exit 3
(cd ab_old && python3 -m rocmdash._build --check) || exit 3
for i in 1 2 3; do
  for arm in old new; do
    dir=.; [[ $arm == old ]] && dir=ab_old
    echo "[ab_lw] $(date +%T) round $i $arm"
    timeout -k 10 300 python3 $dir/tools/bench_long_window.py --windows 1048576,4194304,16777216 --iters 30 \
      --out "$O/${arm}_$i.json" > "$O/${arm}_$i.log" 2>&1 || exit 1
  done
done
python3 - "$O" <<'PY'
import json, sys, glob, statistics, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*_[0-9].json")):
    arm = f.split("/")[-1].split("_")[0]
    for r in json.load(open(f)):
        if r["launch"] == "direct":
            res[(r["W"], r["data"], arm)].append(r["p50_us"])
for (W, data, arm), v in sorted(res.items()):
    print(f"W={W:>9d} {data:10s} {arm}: p50 us per round {v} median {statistics.median(v)}")
PY
