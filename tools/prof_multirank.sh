#!/bin/bash
# Kernel trace of the N > 1 native gather with 2 ranks on one MI355X (oversubscribed:
# RCCL between the ranks over sockets). Rank 1 runs plainly, rank 0 under rocprofv3
# --kernel-trace --stats: RCCL's multi-rank all-gather kernel, the publish kernel and the
# window-stats kernel of every refresh. Both ranks are started from this shell (no
# launcher between the profiler and the program).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r3prof}
mkdir -p $O
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 WORLD_SIZE=2 ROCMDASH_OVERSUBSCRIBE=1 NCCL_DEBUG=WARN
export TMPDIR=/tmp
RANK=1 LOCAL_RANK=1 timeout -k 10 240 python tools/multirank_check.py --refreshes 300 --node-window 0 > $O/rank1.log 2>&1 &
r1=$!
RANK=0 LOCAL_RANK=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
    python tools/multirank_check.py --refreshes 300 --node-window 0 > $O/rank0.log 2>&1
rc0=$?
wait $r1
rc1=$?
echo "rank0 rc=$rc0 rank1 rc=$rc1"
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
test -f $O/kernel_stats.csv && cut -d, -f1-8 $O/kernel_stats.csv | head -20
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ]
