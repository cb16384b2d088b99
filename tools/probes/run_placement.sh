#!/bin/bash
# GPU-box check of the init placement (rocmdash/runtime/placement.py): the bench three
# times with the default (auto: first run calibrates, the others use the cache), then
# once with it off, alternating with auto again.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
show() { python3 -c "import json; d=json.load(open('$1')); print('$2', d['value'], d['ms_per_step'], d['p50_refresh_ms'], d['sampler_p50_us'], d['sampler_threads'], d.get('init_placement'))"; }
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --json-out "$OUT/placement_auto_$i.json" > "$OUT/placement_auto_$i.log" 2>&1 || exit $?
  show "$OUT/placement_auto_$i.json" "auto$i"
done
for i in 1 2; do
  ROCMDASH_INIT_PLACEMENT=0 timeout -k 10 300 python3 bench.py --json-out "$OUT/placement_off_$i.json" > "$OUT/placement_off_$i.log" 2>&1 || exit $?
  show "$OUT/placement_off_$i.json" "off$i"
done
