#!/bin/bash
# GPU-box A/B of the init placement: bench with auto placement vs off, alternating,
# 5 rounds (the first auto run calibrates, later ones use the cache).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
show() { python3 -c "import json; d=json.load(open('$1')); print('$2', d['value'], d['ms_per_step'], d['p50_refresh_ms'], d['sampler_p50_us'], d.get('init_placement'))"; }
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --json-out "$OUT/pab_auto_$i.json" > "$OUT/pab_auto_$i.log" 2>&1 || exit $?
  show "$OUT/pab_auto_$i.json" "auto$i"
  ROCMDASH_INIT_PLACEMENT=0 timeout -k 10 300 python3 bench.py --json-out "$OUT/pab_off_$i.json" > "$OUT/pab_off_$i.log" 2>&1 || exit $?
  show "$OUT/pab_off_$i.json" "off$i"
done
