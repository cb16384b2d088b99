#!/bin/bash
# PMC of the long-window streaming passes at W = 2^24 mixed-sign data: pass B (bracket
# mode, the default) in one run, pass 0 of the radix chain (ROCMDASH_LW_BRACKETS=0) in
# another; per (kernel, grid) the median per dispatch of the SQ instruction / wave-cycle
# counters (one pass, <= 8 SQ + 1 GRBM counters).
# Usage (via gpurun): bash tools/pmc_brackets.sh [out_dir]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_brackets}; mkdir -p "$O"
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
for arm in brackets radix; do
  b=1; [[ $arm == radix ]] && b=0
  ROCMDASH_LW_BRACKETS=$b timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM \
    SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -d "$O/$arm" -o run --output-format csv -- python3 tools/bench_long_window.py --windows 16777216 --shapes normal --iters 10 \
    > "$O/$arm.log" 2>&1 || { tail -5 "$O/$arm.log"; exit 1; }
done
python3 - "$O" <<'PY' | tee "$O/summary.txt"
import csv, sys, glob, collections, statistics
for arm in ("brackets", "radix"):
    f = glob.glob(f"{sys.argv[1]}/{arm}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "lw_pass" not in n:
            continue
        k = n[n.find("lw_pass"):].split("(")[0]
        acc[(k, r.get("Grid_Size", r.get("Grid_Size_X", "")))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (k, g) in sorted(acc):
        d = acc[(k, g)]
        n = len(next(iter(d.values())))
        print(arm, k, "grid", g, "dispatches", n, {c: round(statistics.median(v) / 1e6, 2) for c, v in sorted(d.items())},
              "(M, median per dispatch)")
PY
