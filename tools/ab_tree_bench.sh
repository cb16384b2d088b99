#!/bin/bash
# A/B of bench.py between this tree (new) and the build in .ab_old/ (old), alternating.
# Usage (via gpurun): bash tools/ab_tree_bench.sh ROUNDS [bench args...]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abtree; mkdir -p "$OUT"; export TMPDIR=/tmp
ROUNDS=$1; shift
for r in $(seq 1 "$ROUNDS"); do
  for side in new old; do
    dir=.; [[ $side == old ]] && dir=.ab_old
    (cd "$dir" && timeout -k 10 300 python3 bench.py --steps 2000 --warmup 100 --timing-steps 0 "$@" \
      --json-out "/tmp/abtree_${side}_$r.json") > "$OUT/${side}_$r.log" 2>&1 || { echo "FAIL $side"; tail -5 "$OUT/${side}_$r.log"; exit 1; }
    cp "/tmp/abtree_${side}_$r.json" "$OUT/"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['p50_refresh_ms'], d['value'], d['p50_breakdown_ms'], d['sampler_p50_us'], d.get('startup_restarts'))" "/tmp/abtree_${side}_$r.json" "$side"
  done
done
