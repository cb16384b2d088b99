#!/bin/bash
# GPU-box probe: fast / slow SMU-table read states across fresh processes, idle and
# with the GPU kept busy by another process (probe_state.cpp).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
g++ -O2 -o "$OUT/probe_state" tools/probes/probe_state.cpp || exit 1
echo "== idle GPU, 8 fresh processes"
for i in 1 2 3 4 5 6 7 8; do timeout -k 5 30 "$OUT/probe_state" 2000 || exit $?; done
echo "== GPU busy (bf16 GEMM loop in another process), 8 fresh processes"
timeout -k 5 90 python3 -c "
import torch, time
a = torch.randn(8192, 8192, device='cuda', dtype=torch.bfloat16)
t0 = time.time()
while time.time() - t0 < 60:
    for _ in range(10): a @ a
    torch.cuda.synchronize()
" &
load=$!
sleep 15
for i in 1 2 3 4 5 6 7 8; do timeout -k 5 30 "$OUT/probe_state" 2000 || break; done
kill $load 2>/dev/null
wait $load
echo "== idle again, 4 fresh processes"
for i in 1 2 3 4; do timeout -k 5 30 "$OUT/probe_state" 2000 || exit $?; done
