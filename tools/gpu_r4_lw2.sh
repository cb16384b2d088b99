#!/bin/bash
# Long-window kernel iteration: its GPU tests (incl. the node-window ones), then the A/B.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r4_lw2}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
echo "== $(date +%T) long-window GPU tests"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_long_window.py tests/test_gpu_multirank.py -k "long_window" -x -v \
  --timeout 240 --timeout-method thread > "$OUT/pytest_lw.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_lw.log"; [[ $rc == 0 ]] || exit $rc
echo "== $(date +%T) A/B"
timeout -k 10 400 python3 tools/bench_long_window.py --windows 4194304,16777216 --shapes normal,telemetry \
  --chunks 16384 --wave-private-ab --compact-ab --old-ab --bf-ab --iters 30 --rounds 2 --out "$OUT/lw_ab.json" > "$OUT/lw_ab.log" 2>&1 || exit 1
python3 tools/summarize_lw_ab.py "$OUT/lw_ab.log"
echo "== $(date +%T) kernel trace W = 2^24"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 tools/bench_long_window.py --windows 16777216 --shapes normal,telemetry --iters 20 > "$OUT/trace.log" 2>&1 || exit 1
python3 tools/summarize_prof.py "$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)" --out "$OUT/trace_summary.json" > /dev/null || true
echo "== $(date +%T) done"
