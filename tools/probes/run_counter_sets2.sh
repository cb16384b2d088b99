#!/bin/bash
# Read cost of the current device-counter set vs the same set + one candidate SQ counter
# (alternating, 3 reps). Usage (via gpurun): bash tools/probes/run_counter_sets2.sh
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
C=GRBM_COUNT,GRBM_GUI_ACTIVE,SQ_VALU_MFMA_BUSY_CYCLES,TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum,SQ_BUSY_CU_CYCLES
for rep in 1 2 3; do
  for s in $C $C,SQ_WAVES $C,SQ_INSTS_VALU $C,SQ_INSTS_SALU $C,SQ_INSTS_LDS $C,SQ_WAVES,SQ_INSTS_VALU; do
    timeout -k 10 120 python3 tools/probes/probe_counter_cost.py $s --n 1000 2>/dev/null | grep "{" || exit 1
  done
done
