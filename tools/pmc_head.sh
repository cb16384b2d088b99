#!/bin/bash
# Steady-state stats kernel at HEAD on one box: HIP events around the refresh for each
# completion signal (0 none / 1 flag / 2 tagged), then a rocprofv3 LDS/VALU PMC pass of the
# one-row launch (W = 4096 x 15 series, k = 1). Usage (via gpurun): bash tools/pmc_head.sh
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_head
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
for rep in 1 2; do
  for sig in 1 2 0; do
    timeout -k 10 120 python3 tools/bench_kernel.py --iters 400 --windows 4096 --series 15 --ks 1 10 --signal $sig \
      > "$OUT/events_sig${sig}_$rep.jsonl" 2>"$OUT/events_sig${sig}_$rep.err" || { tail -5 "$OUT/events_sig${sig}_$rep.err"; exit 1; }
    echo "rep $rep signal $sig: $(tr '\n' ' ' < "$OUT/events_sig${sig}_$rep.jsonl")"
  done
done
rm -rf "$OUT/pmc"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS \
  -d "$OUT/pmc" -o pmc --output-format csv \
  -- python3 tools/bench_kernel.py --iters 60 --windows 4096 --series 15 --ks 1 --signal 2 > "$OUT/pmc.log" 2>&1
rc=$?; tail -2 "$OUT/pmc.log"; [[ $rc == 0 ]] || exit $rc
python3 - "$OUT/pmc" <<'PY'
import csv, glob, statistics, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "window_stats_kernel<512, 8>" in r["Kernel_Name"]:
        by[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = collections.defaultdict(list)
for d in by.values():
    for k, v in d.items():
        per[k].append(sum(v))
med = {k: statistics.median(v) for k, v in per.items()}
print("window_stats_kernel<512, 8>, W=4096, 15 series, k=1, tagged outputs; median per dispatch over", len(by), "dispatches:",
      ", ".join(f"{k}={v:.0f}" for k, v in sorted(med.items())),
      "-> bank conflicts %.1f%% of LDS-active cycles" % (100 * med.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, med.get("SQ_LDS_IDX_ACTIVE", 1))))
PY
