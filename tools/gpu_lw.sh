#!/bin/bash
# Long-window / node-window measurements on one MI355X box, one parameterised script
# (replaces the round-4 one-off lease scripts gpu_r4_lw*.sh / gpu_r4_all.sh).
#
#   bash tools/gpu_lw.sh OUTDIR STEP [STEP ...]
#
# Steps (each under its own time limit; the script stops at the first failure):
#   tests        long-window GPU tests (tests/test_gpu_long_window.py)
#   gputests     the whole GPU suite (pytest -m gpu)
#   bench        the driver-shape bench (bench.py --steps 20 --warmup 5)
#   ab           tools/bench_long_window.py A/B: $WINDOWS x $SHAPES with $AB (e.g.
#                "--brackets-ab --chunks 32768", "--prefetch-ab --old-ab --compact-ab",
#                "--wave-private-ab --compact-ab --old-ab --bf-ab --chunks 16384",
#                "--half-wave-ab --brackets-ab --chunks 32768", "--incremental-ab")
#   trace        rocprofv3 kernel trace at 2^24 + per-pass phases
#   layouts      per-pass kernel times for the ring layouts 8+4, 8, 4, 12, 4+4+4
#   pmc          two PMC passes over the passes (instruction mix; LDS conflicts / busy)
#   kernarg      kernel arguments in host (0) vs device (1) memory
#   nodewin      bench.py --node-window at 2^24 with the one-rank communicator
#   nodewintrace the same under a rocprofv3 kernel trace (per-kernel stats)
#   nodecheck    tools/node_long_window_check.py, one rank, 2^22 (collectives timed)
#   nodecheck2 / nodecheck4   the same at 2 / 4 oversubscribed ranks, 2^20
#   idle         HIP idle wake-up probe
#   duty         counter duty-cycle experiment
# Environment: WINDOWS (default 4194304,16777216), SHAPES (normal,telemetry), AB, ITERS (30),
# NODECHECK_ARGS (extra node check arguments, e.g. --full-cap).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:?usage: gpu_lw.sh OUTDIR STEP...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
WINDOWS=${WINDOWS:-4194304,16777216}
SHAPES=${SHAPES:-normal,telemetry}
AB=${AB:-}
ITERS=${ITERS:-30}
NODECHECK_ARGS=${NODECHECK_ARGS:-}
step() { echo "== $(date +%T) $*"; }
fail() { tail -5 "$1"; exit 1; }
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }

phases() {  # per-pass kernel phases from a trace directory
  local f
  f=$(find "$1" -name '*kernel_trace.csv' | head -1 || true)
  [[ -n "$f" ]] && python3 tools/lw_trace_phases.py "$f" 10 > "$2" && cat "$2"
  return 0
}

nodecheck() {  # ranks window tag
  if [[ $1 == 1 ]]; then
    # shellcheck disable=SC2086
    timeout -k 10 300 python3 tools/node_long_window_check.py --window "$2" $NODECHECK_ARGS > "$OUT/$3.json" 2> "$OUT/$3.err" || fail "$OUT/$3.err"
  else
    ROCMDASH_OVERSUBSCRIBE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$1" \
      --master-addr 127.0.0.1 --master-port $((29560 + $1)) tools/node_long_window_check.py --window "$2" \
      --capacity 131072 $NODECHECK_ARGS > "$OUT/$3.json" 2> "$OUT/$3.err" || fail "$OUT/$3.err"
  fi
  grep '^{' "$OUT/$3.json" | tail -1 | cut -c1-900
}

for s in "$@"; do
  step "$s"
  case "$s" in
    tests)
      timeout -k 10 500 python3 -u -m pytest tests/test_gpu_long_window.py -x -v --timeout 240 --timeout-method thread \
        > "$OUT/pytest_lw.log" 2>&1 || fail "$OUT/pytest_lw.log"
      tail -3 "$OUT/pytest_lw.log" ;;
    gputests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || fail "$OUT/pytest_gpu.log"
      tail -3 "$OUT/pytest_gpu.log" ;;
    bench)
      timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --json-out "$OUT/bench_k20.json" \
        > "$OUT/bench_k20.log" 2>&1 || fail "$OUT/bench_k20.log"
      tail -c 300 "$OUT/bench_k20.json" ;;
    ab)
      # shellcheck disable=SC2086
      timeout -k 10 600 python3 tools/bench_long_window.py --windows "$WINDOWS" --shapes "$SHAPES" $AB \
        --iters "$ITERS" --rounds 2 --out "$OUT/lw_ab.json" > "$OUT/lw_ab.log" 2>&1 || fail "$OUT/lw_ab.log"
      python3 tools/summarize_lw_ab.py "$OUT/lw_ab.log" ;;
    trace)
      # shellcheck disable=SC2086
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
        -- python3 tools/bench_long_window.py --windows 16777216 --shapes "$SHAPES" --iters 20 $AB \
        > "$OUT/trace.log" 2>&1 || fail "$OUT/trace.log"
      phases "$OUT/trace" "$OUT/phases.txt" ;;
    layouts)
      for layout in 8+4 8 4 12 4+4+4; do
        tag=${layout//+/_}
        timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$tag" -o run \
          -- python3 tools/bench_long_window.py --windows 16777216 --shapes "$SHAPES" --iters 20 --layout "$layout" \
          > "$OUT/layout_$tag.log" 2>&1 || fail "$OUT/layout_$tag.log"
        phases "$OUT/trace_$tag" "$OUT/phases_$tag.txt"
      done ;;
    pmc)
      for pmc in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
                 "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
        tag=$(echo "$pmc" | cut -d' ' -f1)
        # shellcheck disable=SC2086
        timeout -s KILL 120 rocprofv3 --pmc $pmc -d "$OUT/pmc_$tag" -o run --output-format csv \
          -- python3 tools/bench_long_window.py --windows 16777216 --shapes "$SHAPES" --iters 10 $AB \
          > "$OUT/pmc_$tag.log" 2>&1 || fail "$OUT/pmc_$tag.log"
      done ;;
    kernarg)
      for kd in 0 1; do
        HIP_FORCE_DEV_KERNARG=$kd timeout -k 10 200 python3 tools/bench_long_window.py --windows 16777216 \
          --shapes telemetry --brackets-ab --iters 30 > "$OUT/kernarg_$kd.log" 2>&1 || fail "$OUT/kernarg_$kd.log"
        grep p50_us "$OUT/kernarg_$kd.log" | cut -c1-150
      done ;;
    nodewin)
      timeout -k 10 300 python3 bench.py --window 16777216 --node-window --gather rccl --steps 20 --warmup 3 \
        --timing-steps 0 --e2e-s 0 --prefill 2000 --prefill-generated 16777216 --json-out "$OUT/bench_nodewin_2p24.json" \
        > "$OUT/bench_nodewin_2p24.log" 2>&1 || fail "$OUT/bench_nodewin_2p24.log"
      tail -c 600 "$OUT/bench_nodewin_2p24.json" ;;
    nodewintrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nodewin_trace" -o run \
        -- python3 bench.py --window 16777216 --node-window --gather rccl --steps 20 --warmup 3 --timing-steps 0 \
        --e2e-s 0 --production-s 0 --prefill 2000 --prefill-generated 16777216 --restarts 0 \
        --json-out "$OUT/bench_nodewin_trace.json" > "$OUT/nodewin_trace.log" 2>&1 || fail "$OUT/nodewin_trace.log"
      f=$(find "$OUT/nodewin_trace" -name '*kernel_stats.csv' | head -1 || true)
      [[ -n "$f" ]] && head -30 "$f" ;;
    nodecheck) nodecheck 1 4194304 node_lw_w1_2p22 ;;
    nodecheck2) nodecheck 2 1048576 node_lw_w2_2p20 ;;
    nodecheck4) nodecheck 4 1048576 node_lw_w4_2p20 ;;
    idle)
      timeout -k 10 200 python3 tools/probes/probe_idle_wakeup.py > "$OUT/idle_wakeup.jsonl" 2>&1 || fail "$OUT/idle_wakeup.jsonl"
      cat "$OUT/idle_wakeup.jsonl" ;;
    duty)
      timeout -k 10 200 python3 tools/probes/probe_counter_duty.py --modes 0,200,1000 --seconds 10 \
        > "$OUT/counter_duty.jsonl" 2>&1 || fail "$OUT/counter_duty.jsonl"
      cat "$OUT/counter_duty.jsonl" ;;
    *)
      echo "unknown step $s" >&2
      exit 2 ;;
  esac
done
step done
