#!/bin/bash
# A/B on one MI355X box: the launch configuration for refreshes with at most 2 new rows
# per ring (ROCMDASH_SMALL_K_ROWS=1: <1024, 4> general path for the whole launch as soon
# as one ring brings 2 rows; =2: <512, 8>, one-row path for the 1-row series), 3
# alternating rounds of the default (free-running) N = 1 bench.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r3smallk}; mkdir -p $O
python3 -m rocmdash._build --check || exit 3
for i in 1 2 3; do
  for k in 1 2; do
    echo "[ab_small_k] $(date +%T) round $i k=$k"
    ROCMDASH_SMALL_K_ROWS=$k timeout -k 10 200 python bench.py --steps 4000 --warmup 100 --e2e-s 0 --timing-steps 0 \
        > $O/bench_k$k\_$i.json 2> $O/bench_k$k\_$i.err || exit 1
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["p50_refresh_ms"], d["p90_refresh_ms"], d["ms_per_step"], d["sampler_mean_us"],
          d["p50_breakdown_ms"])
PY
