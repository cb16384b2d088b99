#!/bin/bash
# which counter costs the round-5 read its +27 us. Alternates the
# round-4 6-counter set, round-5's 7, the 7 with RDREQ_sum in place of RDREQ_DRAM_32B,
# the 7 without WRREQ_64B, and the 6-counter candidate whose write bytes come from ONE
# 32 B-unit counter (WRREQ_WRITE_DRAM_32B) - 3 reps each, one process per set, each
# line also carrying the set's byte accuracy against known traffic.
# Usage (via gpurun): bash tools/probes/run_counter_ab.sh OUT_JSONL
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=${1:-gpurun_out/counter_ab.jsonl}
mkdir -p "$(dirname "$out")"
B=GRBM_COUNT,GRBM_GUI_ACTIVE,SQ_VALU_MFMA_BUSY_CYCLES
R4=$B,TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum,SQ_BUSY_CU_CYCLES
R5=$B,TCC_EA0_RDREQ_DRAM_32B_sum,TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum,SQ_BUSY_CU_CYCLES
R5RD=$B,TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum,SQ_BUSY_CU_CYCLES
R5NO64=$B,TCC_EA0_RDREQ_DRAM_32B_sum,TCC_EA0_WRREQ_sum,SQ_BUSY_CU_CYCLES
R6=$B,TCC_EA0_RDREQ_DRAM_32B_sum,TCC_EA0_WRREQ_WRITE_DRAM_32B_sum,SQ_BUSY_CU_CYCLES
# one placement decision for every process (the A/B must not mix NUMA states, nor pay a
# re-probe per process while the calibration reads "slow")
node=$(timeout -k 10 300 python3 -c "
import json
from rocmdash.runtime import placement, topology
d = placement.calibrate(0, topology.bdf_of_hip_device(0) or 0, use_cache=False)
print(json.dumps(d), file=open('$out.placement.json', 'w'))
print(d.get('node') if d.get('node') is not None else 0)
") || exit 1
export ROCMDASH_INIT_PLACEMENT=$node
for rep in 1 2 3; do
  for s in $R4 $R5 $R5RD $R5NO64 $R6; do
    timeout -k 10 120 python3 -u tools/probes/probe_counter_accuracy.py $s --n 1000 2>>"$out.err" | grep "{" >> "$out" || exit 1
  done
done
