#!/bin/bash
# How often does a fresh bench process land in the slow counter-read state, by when the
# init pin is released (ROCMDASH_RESTORE_AT=init|end) and where the sampler threads run
# (ROCMDASH_PIN_SAMPLERS)? Alternating configurations, no restarts, short runs.
# (ROCMDASH_RESTORE_AT was an experiment-only switch in GpuAgent, removed after this run:
# profiles/r02/state_ab.txt.) Usage: bash tools/probes/run_state_ab.sh ROUNDS
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/state_ab; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 "${1:-6}"); do
  for cfg in "init|ROCMDASH_RESTORE_AT=init" "end|ROCMDASH_RESTORE_AT=end" "end_nopin|ROCMDASH_RESTORE_AT=end ROCMDASH_PIN_SAMPLERS=off"; do
    label=${cfg%%|*}; read -r -a envs <<< "${cfg#*|}"
    env "${envs[@]}" ROCMDASH_BENCH_RESTARTS=0 timeout -k 10 120 python3 bench.py --steps 300 --warmup 20 --timing-steps 0 \
      --json-out "$OUT/${label}_$r.json" > "$OUT/${label}_$r.log" 2>&1 || { echo "FAIL $label"; tail -3 "$OUT/${label}_$r.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['sampler_p50_us'], d['ms_per_step'], d['init_placement'].get('node') if d['init_placement'] else None, d['sampler_threads'])" "$OUT/${label}_$r.json" "$label"
  done
done
