#!/bin/bash
# The driver's situation: bench.py as the FIRST process on a fresh box (calibration and
# the measurement may land in the box-wide slow phase right after start-up), then again.
# Usage (via gpurun): bash tools/fresh_box_bench.sh [REPS]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fresh_box
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 "${1:-3}"); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out "$OUT/bench_$r.json" > "$OUT/bench_$r.log" 2>&1 \
    || { tail -5 "$OUT/bench_$r.log"; exit 1; }
  grep "slow driver state" "$OUT/bench_$r.log" | cut -c1-200
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['p50_refresh_ms'], 'restarts', d['startup_restarts'], 'settle_s', d.get('settle_s'), d['init_placement'], d['sampler_p50_us'])" "$OUT/bench_$r.json" "run$r"
done
