set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r5_pmc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_long_window.py --windows 16777216 --shapes normal --new-rows 100 --iters 30 --chunks 4096,8192 > $OUT/chunks.log 2>&1 || { tail -5 $OUT/chunks.log; exit 1; }
grep p50_us $OUT/chunks.log | cut -c1-200
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS -d "$GRAFT_REPO_ROOT/$OUT/pmc1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_long_window.py" --windows 16777216 --shapes normal --new-rows 100 --iters 10 > "$GRAFT_REPO_ROOT/$OUT/pmc1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACCUM_PREV_HIRES GRBM_GUI_ACTIVE GRBM_COUNT -d "$GRAFT_REPO_ROOT/$OUT/pmc2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_long_window.py" --windows 16777216 --shapes normal --new-rows 100 --iters 10 > "$GRAFT_REPO_ROOT/$OUT/pmc2.log" 2>&1 || exit 1
echo done
