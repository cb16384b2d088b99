#!/bin/bash
# One gpurun call: GPU tests, the driver-shape bench, then the long-window / node-window /
# counter-duty measurements (tools/gpu_r4_lw.sh). Stops at the first failing step.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r4}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
echo "== $(date +%T) pytest -m gpu"
timeout -k 10 720 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [[ $rc == 0 ]] || exit $rc
echo "== $(date +%T) bench (driver shape)"
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --json-out "$OUT/bench_k20.json" > "$OUT/bench_k20.log" 2>&1
rc=$?; tail -c 300 "$OUT/bench_k20.json"; [[ $rc == 0 ]] || exit $rc
bash tools/gpu_r4_lw.sh "$OUT/lw"
