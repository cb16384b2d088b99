#!/bin/bash
# PMC of the long-window passes, v3 worktree (./ab_old) vs this tree, W = 2^24 mixed-sign
# data (one pass per counter set; SQ counters only, <= 8 per pass).
# Usage (via gpurun): bash tools/pmc_long_window_ab.sh [out_dir]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/lwpmc}; mkdir -p "$O"
for arm in old new; do
  dir=.; [[ $arm == old ]] && dir=ab_old
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    -d "$O/$arm" -o run --output-format csv -- python3 $dir/tools/bench_long_window.py --windows 16777216 --shapes normal --iters 5 \
    > "$O/$arm.log" 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import csv, sys, glob, collections, statistics
for arm in ("old", "new"):
    f = glob.glob(f"{sys.argv[1]}/{arm}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "lw_pass" not in n:
            continue
        k = n[n.find("lw_pass"):n.find("lw_pass") + 10]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        print(arm, k, {c: round(statistics.median(v) / 1e6, 2) for c, v in sorted(acc[k].items())}, "(M, median per dispatch)")
PY
