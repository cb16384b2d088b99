B=GRBM_COUNT,GRBM_GUI_ACTIVE,SQ_VALU_MFMA_BUSY_CYCLES,TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum
for rep in 1 2; do
for s in $B $B,SQ_BUSY_CU_CYCLES $B,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES $B,SQ_BUSY_CU_CYCLES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES $B,SQ_WAVES $B,SQ_INSTS_VALU; do
  timeout -k 10 120 python3 tools/probes/probe_counter_cost.py $s 2>/dev/null | grep "{" || exit 1
done; done
