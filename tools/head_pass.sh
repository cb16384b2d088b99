#!/bin/bash
# The round's HEAD measurement pass on one MI355X box (results copied to profiles/<round>/head/):
# GPU tests, smoke, headline bench x3 (+ extended, closed-loop, serial, one-rank native RCCL path),
# rocprofv3 kernel trace of the headline bench, multi-rank native gather on this GPU (+ its
# kernel trace), the exporter's footprint, deployed-path e2e (manifests and fast configs).
# Usage (via gpurun, from the repo root): bash tools/head_pass.sh [outdir] [a|b|all]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/head}
PART=${2:-all}  # a: tests, smoke, benches, headline trace; b: multi-rank, footprint, e2e
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }

if [[ $PART != b ]]; then
step pytest -m gpu
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [[ $rc == 0 ]] || exit $rc
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/smoke.log" | tail -4; [[ $rc == 0 ]] || exit $rc
for cfg in "bench_n1|" "bench_n1_2|" "bench_n1_3|" "bench_n1_extended|--extended" "bench_n1_closed|--sampling closed" "bench_n1_serial|--sampling closed --prefetch 0" "bench_n1_rccl|--gather rccl"; do
  name=${cfg%%|*}; args=${cfg#*|}
  step "bench $name $args"
  timeout -k 10 300 python3 bench.py $args --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
  rc=$?; tail -1 "$OUT/$name.log" | cut -c1-160; [[ $rc == 0 ]] || exit $rc
done
step "rocprofv3 kernel trace of the headline bench (device counters off under the profiler)"
rm -rf "$OUT/prof"
ROCMDASH_COUNTERS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 bench.py --steps 300 --warmup 20 --timing-steps 0 > "$OUT/prof.log" 2>&1
rc=$?; tail -1 "$OUT/prof.log" | cut -c1-160; [[ $rc == 0 ]] || exit $rc
python3 tools/summarize_prof.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" --out "$OUT/headline_profile.json" || exit 1
fi
if [[ $PART != a ]]; then
step "multi-rank native gather on this GPU (2 and 4 oversubscribed ranks) + kernel trace"
for n in 2 4; do
  ROCMDASH_OVERSUBSCRIBE=1 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29700 + n)) tools/multirank_check.py --refreshes 60 > "$OUT/multirank_$n.log" 2>&1
  rc=$?; grep '^{' "$OUT/multirank_$n.log" > "$OUT/multirank_$n.json"; [[ $rc == 0 ]] || exit $rc
done
bash tools/prof_multirank.sh "$OUT/multirank_prof" > "$OUT/multirank_prof.log" 2>&1 || exit 1
python3 tools/summarize_rocpd.py "$OUT/multirank_prof/prof/run_results.db" --csv "$OUT/multirank_kernel_stats.csv" > /dev/null || exit 1
step "footprint at production rates (world 1, live sources)"
timeout -k 10 300 python3 tools/footprint_probe.py --world 1 --seconds 10 --out "$OUT/footprint_w1.json" > "$OUT/footprint_w1.log" 2>&1 || exit 1
step "e2e: DaemonSet config (from the manifests), then fast config"
timeout -k 10 300 python3 tools/bench_e2e.py --manifests deploy/k8s --seconds 30 --out "$OUT/e2e_daemonset.json" > "$OUT/e2e_daemonset.log" 2>&1
rc=$?; tail -2 "$OUT/e2e_daemonset.log" | cut -c1-200; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python3 tools/bench_e2e.py --seconds 30 --refresh-hz 10 --scrape-s 0.25 --page-s 0.5 --out "$OUT/e2e_fast.json" > "$OUT/e2e_fast.log" 2>&1
rc=$?; tail -2 "$OUT/e2e_fast.log" | cut -c1-200; [[ $rc == 0 ]] || exit $rc
step "e2e: 8 service ranks on this GPU (oversubscribed) from the manifests"
timeout -k 10 300 python3 tools/bench_e2e.py --manifests deploy/k8s --world 8 --seconds 20 --out "$OUT/e2e_manifests_8rank.json" > "$OUT/e2e_manifests_8rank.log" 2>&1
rc=$?; tail -2 "$OUT/e2e_manifests_8rank.log" | cut -c1-200; [[ $rc == 0 ]] || exit $rc
fi
step done
