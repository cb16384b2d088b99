#!/bin/bash
# Round-3 GPU pass (one MI355X box): GPU tests, multi-rank native gather on one GPU,
# the headline bench, the deployed path as the manifests ship it, the exporter's own
# footprint, the placement calibration's cost, then the native-gather rank-loss test.
# Every step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3
mkdir -p $O
export PYTHONUNBUFFERED=1
step() { echo "[gpu_round3] $(date +%T) $*"; }

step pytest-gpu && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "not recovers_from_rank_loss" > $O/pytest_gpu.txt 2>&1 && tail -3 $O/pytest_gpu.txt &&
for n in 2 4 8; do
  step multirank $n && ROCMDASH_OVERSUBSCRIBE=1 NCCL_DEBUG=WARN timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) tools/multirank_check.py --refreshes 60 \
      > $O/multirank_$n.log 2>&1 && grep '^{' $O/multirank_$n.log > $O/multirank_$n.json || exit 1
done &&
step bench-n1 && timeout -k 10 300 python bench.py --steps 2000 --warmup 100 > $O/bench_n1.json 2> $O/bench_n1.err &&
step bench-n1-rccl && timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --gather rccl > $O/bench_n1_rccl.json 2> $O/bench_n1_rccl.err &&
step e2e-manifests && timeout -k 10 300 python tools/bench_e2e.py --manifests deploy/k8s --seconds 20 --out $O/e2e_daemonset_manifests.json > $O/e2e.log 2>&1 &&
step footprint-1 && timeout -k 10 300 python tools/footprint_probe.py --world 1 --seconds 10 --out $O/footprint_w1.json > $O/footprint_w1.log 2>&1 &&
step footprint-4 && timeout -k 10 300 python tools/footprint_probe.py --world 4 --counters synthetic --seconds 10 --out $O/footprint_w4.json > $O/footprint_w4.log 2>&1 &&
step placement && timeout -k 10 300 python -c "
import json, time
from rocmdash.runtime import placement as p
t = time.perf_counter()
tab = p._probe_all(p.numa_nodes(), '/tmp/rocmdash_cal_probe.json')
tab['wall_s'] = round(time.perf_counter() - t, 2)
print(json.dumps(tab))" > $O/placement_probe_all.json 2> $O/placement.err &&
step serve-rank-loss && timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread \
    -k "recovers_from_rank_loss" > $O/pytest_rank_loss.txt 2>&1 && tail -3 $O/pytest_rank_loss.txt &&
step done
