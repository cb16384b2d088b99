#!/bin/bash
# A/B on one box: SMU metrics-table reads on every refresh (0) vs at most every 2 ms
# (ROCMDASH_SMU_TABLE_MIN_US=2000; used VRAM still read live every refresh), 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r3smu}; mkdir -p $O
for i in 1 2 3; do
  for v in 0 2000; do
    echo "[ab_smu] $(date +%T) round $i min_us=$v"
    ROCMDASH_SMU_TABLE_MIN_US=$v timeout -k 10 200 python bench.py --steps 4000 --warmup 100 --e2e-s 0 --timing-steps 0 \
        > $O/bench_$v\_$i.json 2> $O/bench_$v\_$i.err || exit 1
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["p50_refresh_ms"], d["ms_per_step"], d["sampler_p50_us"], d["sampler_mean_us"],
          d["smi_table_refreshes_per_s"], d["smu_table_reads_per_s"])
PY
