#!/bin/bash
# Long-window pass 0 with an LDS histogram copy per half wave (wave_private_level 2): GPU
# tests, A/B against a copy per wave (the default) and uniform 32768-row chunks.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r4_lw9}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
echo "== $(date +%T) long-window GPU tests"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_long_window.py -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_lw.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_lw.log"; [[ $rc == 0 ]] || exit $rc
echo "== $(date +%T) A/B"
timeout -k 10 500 python3 tools/bench_long_window.py --windows 4194304,16777216 --shapes normal,telemetry \
  --half-wave-ab --brackets-ab --chunks 32768 --iters 30 --rounds 2 --out "$OUT/lw_ab.json" > "$OUT/lw_ab.log" 2>&1 || { tail -5 "$OUT/lw_ab.log"; exit 1; }
python3 tools/summarize_lw_ab.py "$OUT/lw_ab.log"
echo "== $(date +%T) done"
