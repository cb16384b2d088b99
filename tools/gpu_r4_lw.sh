#!/bin/bash
# Round-4 long-window / node-window / counter-duty measurements on one MI355X box.
# Usage (via gpurun, from the repo root): bash tools/gpu_r4_lw.sh <outdir>
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r4_lw}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*"; }
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
step "long-window chunk A/B (W = 2^22, 2^24; normal, telemetry)"
timeout -k 10 400 python3 tools/bench_long_window.py --windows 4194304,16777216 --shapes normal,telemetry \
  --chunks 16384 --wave-private-ab --compact-ab --old-ab --bf-ab --iters 30 --rounds 2 --out "$OUT/lw_chunks.json" > "$OUT/lw_chunks.log" 2>&1 || exit 1
tail -2 "$OUT/lw_chunks.log"
step "kernel trace, W = 2^24 normal (auto chunks)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 tools/bench_long_window.py --windows 16777216 --shapes normal,telemetry --iters 20 > "$OUT/trace.log" 2>&1 || exit 1
python3 tools/summarize_prof.py "$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)" --out "$OUT/trace_summary.json" > /dev/null || true
step "node window: bench --node-window at W = 2^24 with the one-rank communicator (collectives timed)"
timeout -k 10 300 python3 bench.py --window 16777216 --node-window --gather rccl --steps 20 --warmup 3 --timing-steps 0 \
  --e2e-s 0 --prefill 2000 --prefill-generated 16777216 --json-out "$OUT/bench_nodewin_2p24.json" > "$OUT/bench_nodewin_2p24.log" 2>&1 || exit 1
tail -c 400 "$OUT/bench_nodewin_2p24.json"
step "node long-window check, one-rank communicator, W = 2^22 (collective steps timed)"
timeout -k 10 300 python3 tools/node_long_window_check.py --window 4194304 > "$OUT/node_lw_w1_2p22.json" 2> "$OUT/node_lw_w1_2p22.err" || exit 1
tail -c 600 "$OUT/node_lw_w1_2p22.json"
step "idle wake-up: kernel event time vs the GPU's idle gap before it"
timeout -k 10 200 python3 tools/probes/probe_idle_wakeup.py > "$OUT/idle_wakeup.jsonl" 2>&1 || exit 1
cat "$OUT/idle_wakeup.jsonl"
step "counter duty-cycle experiment (service rates, 10 s per mode)"
timeout -k 10 200 python3 tools/probes/probe_counter_duty.py --modes 0,200,1000 --seconds 10 > "$OUT/counter_duty.jsonl" 2>&1 || exit 1
cat "$OUT/counter_duty.jsonl"
step done
