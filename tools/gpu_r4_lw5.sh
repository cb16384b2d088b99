#!/bin/bash
# Long-window bracket mode: GPU tests, A/B against the radix chain alone and against
# uniform 32768-row chunks, per-pass kernel times.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r4_lw5}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
echo "== $(date +%T) long-window GPU tests"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_long_window.py -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_lw.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_lw.log"; [[ $rc == 0 ]] || exit $rc
echo "== $(date +%T) A/B"
timeout -k 10 500 python3 tools/bench_long_window.py --windows 1048576,4194304,16777216 --shapes normal,positive,telemetry \
  --brackets-ab --chunks 32768 --iters 30 --rounds 2 --out "$OUT/lw_ab.json" > "$OUT/lw_ab.log" 2>&1 || { tail -5 "$OUT/lw_ab.log"; exit 1; }
python3 tools/summarize_lw_ab.py "$OUT/lw_ab.log"
grep bracket_hits "$OUT/lw_ab.log" | cut -c1-200
for kd in 0 1; do  # kernel arguments in host (0) or device (1) memory: the fixed cost of a launch
  echo "== $(date +%T) HIP_FORCE_DEV_KERNARG=$kd"
  HIP_FORCE_DEV_KERNARG=$kd timeout -k 10 200 python3 tools/bench_long_window.py --windows 16777216 --shapes telemetry \
    --brackets-ab --iters 30 > "$OUT/kernarg_$kd.log" 2>&1 || { tail -5 "$OUT/kernarg_$kd.log"; exit 1; }
  grep p50_us "$OUT/kernarg_$kd.log" | cut -c1-150
done
echo "== $(date +%T) kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run \
  -- python3 tools/bench_long_window.py --windows 16777216 --shapes telemetry,normal --iters 20 --brackets-ab \
  > "$OUT/trace.log" 2>&1 || { tail -5 "$OUT/trace.log"; exit 1; }
f=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1 || true)
[[ -n "$f" ]] && python3 tools/lw_trace_phases.py "$f" 10 | tee "$OUT/phases.txt"
echo "== $(date +%T) done"
