#!/bin/bash
# A/B of the host-out completion signal on one box, alternating: the last-workgroup
# completion flag (ROCMDASH_TAGGED_OUT=0) vs tagged output words (default). Per round:
# a rocprofv3 kernel trace of the headline bench (stats kernel duration) and a bench run
# (refresh p50, device+gather). Usage (via gpurun): bash tools/ab_signal.sh ROUNDS
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_signal
mkdir -p "$OUT"
export TMPDIR=/tmp
ROUNDS=${1:-2}
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
for r in $(seq 1 "$ROUNDS"); do
  for mode in flag:0 tagged:1; do
    label=${mode%%:*}; val=${mode#*:}
    rm -rf "$OUT/prof_${label}_$r"
    ROCMDASH_TAGGED_OUT=$val ROCMDASH_COUNTERS=0 timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/prof_${label}_$r" \
      -o run --output-format csv -- python3 bench.py --steps 1000 --warmup 50 --timing-steps 0 \
      > "$OUT/prof_${label}_$r.log" 2>&1 || { echo "FAIL prof $label"; tail -5 "$OUT/prof_${label}_$r.log"; exit 1; }
    python3 tools/summarize_prof.py "$(find "$OUT/prof_${label}_$r" -name '*kernel_trace.csv' | head -1)" \
      --out "$OUT/trace_${label}_$r.json" > /dev/null || exit 1
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))['kernels']
for k,v in d.items():
    if 'window_stats' in k: print(sys.argv[2], 'trace', k[:40], v['dispatches'], 'p10/p50/p90', v['p10_us'], v['p50_us'], v['p90_us'])
" "$OUT/trace_${label}_$r.json" "$label"
    ROCMDASH_TAGGED_OUT=$val timeout -k 10 180 python3 bench.py --steps 2000 --warmup 100 --timing-steps 0 \
      --json-out "$OUT/bench_${label}_$r.json" > "$OUT/bench_${label}_$r.log" 2>&1 || { echo "FAIL bench $label"; tail -5 "$OUT/bench_${label}_$r.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'bench', d['value'], d['p50_refresh_ms'], d['p90_refresh_ms'], d['p50_breakdown_ms'])" "$OUT/bench_${label}_$r.json" "$label"
  done
done
