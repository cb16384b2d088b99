#!/bin/bash
# A/B of bench.py configurations on one box, alternating, N rounds.
# Usage: bash tools/ab_env.sh ROUNDS "label1|ENV=.. ARGS" "label2|ENV=.. ARGS" ...
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p "$OUT"
export TMPDIR=/tmp
ROUNDS=$1; shift
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    label=${spec%%|*}; rest=${spec#*|}
    envs=(); args=()
    for w in $rest; do if [[ $w == *=* && $w != --* ]]; then envs+=("$w"); else args+=("$w"); fi; done
    env "${envs[@]}" timeout -k 10 180 python3 bench.py --steps 2000 --warmup 100 --timing-steps 0 "${args[@]}" \
      --json-out "$OUT/${label}_$r.json" > "$OUT/${label}_$r.log" 2>&1 || { echo "FAIL $label"; tail -5 "$OUT/${label}_$r.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['p50_refresh_ms'], d['hardware_reads_per_s'], d['value'], d['p50_breakdown_ms'], d['sampler_p50_us'])" "$OUT/${label}_$r.json" "$label"
  done
done
