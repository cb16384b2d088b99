#!/bin/bash
# Round-6 GPU steps (via gpurun): bash tools/gpu_r6.sh OUT step [step ...]
#   procvram   per-process device memory sources (tools/probes/probe_proc_vram.py)
#   queue      the stats stage behind a long-window radix chain, 1 vs 4 hardware queues
#   nodewin    bench.py --node-window at 2^24, 200 node refreshes, twice (VERDICT r05 item 5;
#              round 6's first runs also A/B'd the node-fused records kernel, since removed)
#   nodewin1   the same, off only, once
#   lean8      8 oversubscribed ranks, node-window all-gather of 15 x 4096 samples per rank,
#              default vs the supervisor's lean RCCL environment
#   node8      the production node service on 8 oversubscribed ranks, measured from outside
#   rankvram   per-rank device memory at world 1 / 2 / 8 by start-up stage (lean env)
#   rcclenv    a rank's device memory at world 2 under RCCL settings (MSCCL off, protocols, FIFO)
#   trace      rocprofv3 kernel trace + stats of the driver-shape bench and of the 2^24 node window
#   bench3     the driver-shape bench three times
#   hsaenv     HSA runtime knobs vs a process's driver-side device memory
#   smoke      __graft_entry__.smoke()
#   soak       the supervised node service (counter lanes, 2^20 long window, node window) for 4 minutes
#   soak15     the same soak for 15 minutes with a 2^22 window
#   gputests   the whole GPU test suite
#   bench      the driver-shape bench (python3 bench.py --gpus 1 --steps 20 --warmup 5)
# Every step has its own time limit; the first failure ends the script.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:?out dir}
shift
mkdir -p "$OUT"
fail() { echo "FAILED: $1"; tail -40 "$1"; exit 1; }
NW="--window 16777216 --node-window --gather rccl --steps 200 --warmup 10 --timing-steps 0 --e2e-s 0 --prefill 2000 --prefill-generated 16777216 --production-s 0"
for step in "$@"; do
  case "$step" in
    procvram)
      timeout -k 10 240 python3 -u tools/probes/probe_proc_vram.py "$OUT/proc_vram.json" > "$OUT/proc_vram.log" 2>&1 \
        || fail "$OUT/proc_vram.log" ;;
    queue)
      GPU_MAX_HW_QUEUES=1 timeout -k 10 240 python3 -u tools/probes/probe_queue_contention.py > "$OUT/queue_1.json" \
        2> "$OUT/queue_1.err" || fail "$OUT/queue_1.err"
      timeout -k 10 240 python3 -u tools/probes/probe_queue_contention.py > "$OUT/queue_default.json" \
        2> "$OUT/queue_default.err" || fail "$OUT/queue_default.err" ;;
    nodewin)
      for i in 1 2; do
        timeout -k 10 300 python3 -u bench.py $NW --json-out "$OUT/nodewin_$i.json" > "$OUT/nodewin_$i.log" 2>&1 \
          || fail "$OUT/nodewin_$i.log"
      done ;;
    nodewin1)
      timeout -k 10 300 python3 -u bench.py $NW --json-out "$OUT/nodewin.json" > "$OUT/nodewin.log" 2>&1 \
        || fail "$OUT/nodewin.log" ;;
    lean8)
      for mode in default lean; do
        if [ $mode = lean ]; then E="NCCL_MAX_NCHANNELS=2 NCCL_BUFFSIZE=1048576 GPU_MAX_HW_QUEUES=1 HSA_SCRATCH_SINGLE_LIMIT=1048576"; else E=""; fi
        env $E ROCMDASH_OVERSUBSCRIBE=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) tools/multirank_check.py \
          --refreshes 20 --window 4096 --node-window-reps 50 > "$OUT/lean8_$mode.log" 2>&1 || fail "$OUT/lean8_$mode.log"
        grep "^{" "$OUT/lean8_$mode.log" > "$OUT/lean8_$mode.json" || true
      done ;;
    node8)
      ROCMDASH_OVERSUBSCRIBE=1 timeout -k 10 600 python3 -u tools/node_cpu_probe.py --nproc 8 --seconds 10 \
        --out "$OUT/node8_daemon.json" > "$OUT/node8.log" 2>&1 || fail "$OUT/node8.log" ;;
    rankvram)
      for n in 1 2 8; do
        env GPU_MAX_HW_QUEUES=1 HSA_SCRATCH_SINGLE_LIMIT=1048576 NCCL_BUFFSIZE=1048576 NCCL_MAX_NCHANNELS=2 \
          ROCMDASH_OVERSUBSCRIBE=1 timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 \
          --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29900 + RANDOM % 90)) \
          tools/probes/probe_rank_vram_world.py > "$OUT/rankvram_w$n.log" 2>&1 || fail "$OUT/rankvram_w$n.log"
        grep "^{" "$OUT/rankvram_w$n.log" > "$OUT/rankvram_w$n.jsonl" || true
      done ;;
    rcclenv)
      # which RCCL settings shrink a rank's device memory (world 2, lean environment)
      L="GPU_MAX_HW_QUEUES=1 HSA_SCRATCH_SINGLE_LIMIT=1048576 NCCL_BUFFSIZE=1048576 NCCL_MAX_NCHANNELS=2"
      i=0
      for V in "" "RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0" "NCCL_PROTO=LL,Simple" "NCCL_PROTO=LL" \
               "RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 NCCL_PROTO=LL NCCL_WORK_FIFO_BYTES=65536"; do
        i=$((i + 1))
        echo "$V" > "$OUT/rcclenv_$i.env"
        env $L $V ROCMDASH_OVERSUBSCRIBE=1 timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29800 + RANDOM % 90)) \
          tools/probes/probe_rank_vram_world.py > "$OUT/rcclenv_$i.log" 2>&1 || fail "$OUT/rcclenv_$i.log"
        grep "^{" "$OUT/rcclenv_$i.log" > "$OUT/rcclenv_$i.jsonl" || true
      done ;;
    trace)
      # per-kernel times on the final tree (device counters off: rocprofv3 owns the tool slot)
      ROCMDASH_COUNTERS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_bench" \
        -o run -- python3 -u bench.py --gpus 1 --steps 300 --warmup 20 --production-s 0 --restarts 0 --e2e-s 0 \
        --json-out "$OUT/trace_bench.json" > "$OUT/trace_bench.log" 2>&1 || fail "$OUT/trace_bench.log"
      ROCMDASH_COUNTERS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_nodewin" \
        -o run -- python3 -u bench.py $NW --restarts 0 --json-out "$OUT/trace_nodewin.json" \
        > "$OUT/trace_nodewin.log" 2>&1 || fail "$OUT/trace_nodewin.log" ;;
    bench3)
      for i in 1 2 3; do
        timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_k20_$i.json" \
          2> "$OUT/bench_k20_$i.err" || fail "$OUT/bench_k20_$i.err"
      done ;;
    hsaenv)
      timeout -k 10 300 python3 -u tools/probes/probe_hsa_env.py "$OUT/hsa_env.jsonl" > "$OUT/hsa_env.log" 2>&1 \
        || fail "$OUT/hsa_env.log" ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || fail "$OUT/smoke.log" ;;
    soak)
      timeout -k 10 480 python3 -u tools/soak_node.py --seconds 240 --out "$OUT/soak_node.json" > "$OUT/soak_node.log" \
        2>&1 || fail "$OUT/soak_node.log" ;;
    soak15)
      timeout -k 10 1150 python3 -u tools/soak_node.py --seconds 900 --window 4194304 --out "$OUT/soak15_node.json" \
        > "$OUT/soak15_node.log" 2>&1 || fail "$OUT/soak15_node.log" ;;
    gputests)
      timeout -k 10 1100 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests -m gpu \
        > "$OUT/pytest_gpu.log" 2>&1 || fail "$OUT/pytest_gpu.log" ;;
    bench)
      timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_k20.json" \
        2> "$OUT/bench_k20.err" || fail "$OUT/bench_k20.err" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "done: $step"
done
