#!/bin/bash
# Long-window pass-0 variants: GPU tests, A/B, then PMC of pass 0 on telemetry at 2^24.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r4_lw3}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
echo "== $(date +%T) long-window GPU tests"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_long_window.py -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_lw.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_lw.log"; [[ $rc == 0 ]] || exit $rc
echo "== $(date +%T) A/B"
timeout -k 10 400 python3 tools/bench_long_window.py --windows 4194304,16777216 --shapes normal,telemetry \
  --prefetch-ab --old-ab --compact-ab --iters 30 --rounds 2 --out "$OUT/lw_ab.json" > "$OUT/lw_ab.log" 2>&1 || exit 1
python3 tools/summarize_lw_ab.py "$OUT/lw_ab.log"
for pmc in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  echo "== $(date +%T) pmc $tag"
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d "$OUT/pmc_$tag" -o run --output-format csv \
    -- python3 tools/bench_long_window.py --windows 16777216 --shapes telemetry,normal --iters 10 > "$OUT/pmc_$tag.log" 2>&1 || exit 1
done
echo "== $(date +%T) done"
