#!/bin/bash
# One GPU-box session: probes, GPU tests, 1-GPU bench, rocprofv3 kernel-trace profile.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh [tests|bench|prof|all]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
WHAT=${1:-all}
export TMPDIR=/tmp

step() { echo "== $(date +%T) $*"; }

# the in-tree extension travels with the snapshot: refuse to measure a stale build
python3 -m rocmdash._build --check || { echo "stale native build: run python -m rocmdash._build before gpurun"; exit 3; }

if [[ $WHAT == all || $WHAT == probe ]]; then
  step probe
  timeout -k 10 120 python3 -c "
import torch; p = torch.cuda.get_device_properties(0)
print(torch.__version__, p.name, p.gcnArchName, p.multi_processor_count, round(p.total_memory / 2**30, 1), 'GiB')
" > "$OUT/probe_torch.txt" 2>&1 || exit $?
  cat "$OUT/probe_torch.txt"
fi

if [[ $WHAT == all || $WHAT == tests ]]; then
  step pytest -m gpu
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -25 "$OUT/pytest_gpu.log"; [[ $rc == 0 ]] || exit $rc
fi

if [[ $WHAT == all || $WHAT == bench ]]; then
  step bench
  timeout -k 10 600 python3 bench.py --json-out "$OUT/bench_n1.json" > "$OUT/bench_n1.log" 2>&1
  rc=$?; tail -3 "$OUT/bench_n1.log"; [[ $rc == 0 ]] || exit $rc
  timeout -k 10 600 python3 bench.py --prefetch 0 --json-out "$OUT/bench_n1_serial.json" > "$OUT/bench_n1_serial.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_n1_serial.log"; [[ $rc == 0 ]] || exit $rc
  timeout -k 10 600 python3 bench.py --extended --json-out "$OUT/bench_n1_extended.json" > "$OUT/bench_n1_extended.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_n1_extended.log"; [[ $rc == 0 ]] || exit $rc
fi

if [[ $WHAT == all || $WHAT == prof ]]; then
  step rocprofv3 kernel-trace
  export ROCMDASH_COUNTERS=0  # rocprofv3 owns the profiling tool slot in this run
  rm -rf "$OUT/prof"
  timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 bench.py --steps 300 --warmup 20 > "$OUT/prof.log" 2>&1
  rc=$?; tail -3 "$OUT/prof.log"; [[ $rc == 0 ]] || exit $rc
  find "$OUT/prof" -name '*stats*.csv' | head -5
fi
if [[ $WHAT == prof_rccl ]]; then
  step "rocprofv3 kernel-trace: one-rank RCCL all-gather next to the window-stats kernel (15 series)"
  rm -rf "$OUT/prof_rccl"
  # counters stay on (15 series) unless rocprofv3 and the device-counting tool collide
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rccl" -o run --output-format csv \
    -- python3 bench.py --steps 300 --warmup 20 --gather rccl --timing-steps 0 > "$OUT/prof_rccl.log" 2>&1
  rc=$?; tail -3 "$OUT/prof_rccl.log"; [[ $rc == 0 ]] || exit $rc
  find "$OUT/prof_rccl" -name '*stats*.csv' | head -5
fi
if [[ $WHAT == all || $WHAT == kernel ]]; then
  step kernel micro-benchmark
  timeout -k 10 600 python3 tools/bench_kernel.py --out "$OUT/bench_kernel.json" > "$OUT/bench_kernel.log" 2>&1
  rc=$?; tail -20 "$OUT/bench_kernel.log"; [[ $rc == 0 ]] || exit $rc
  step rocprofv3 kernel-trace of the micro-benchmark
  rm -rf "$OUT/prof_kernel"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_kernel" -o run --output-format csv \
    -- python3 tools/bench_kernel.py --iters 50 --windows 4096 > "$OUT/prof_kernel.log" 2>&1
  rc=$?; tail -3 "$OUT/prof_kernel.log"; [[ $rc == 0 ]] || exit $rc
  step rocprofv3 PMC: LDS / wave counters
  rm -rf "$OUT/pmc_kernel"
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    -d "$OUT/pmc_kernel" -o pmc --output-format csv \
    -- python3 tools/bench_kernel.py --iters 20 --windows 4096 --series 12 > "$OUT/pmc_kernel.log" 2>&1
  rc=$?; tail -3 "$OUT/pmc_kernel.log"; [[ $rc == 0 ]] || exit $rc
fi

if [[ $WHAT == all || $WHAT == smi ]]; then
  step amd-smi latency probe
  hipcc -O2 -o /tmp/probe_smi tools/probes/probe_smi_latency.cpp -I/opt/rocm/include -L/opt/rocm/lib -lamd_smi -Wl,-rpath,/opt/rocm/lib \
    && timeout -k 10 300 /tmp/probe_smi > "$OUT/probe_smi_latency.txt" 2>&1
  rc=$?; cat "$OUT/probe_smi_latency.txt"; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == all || $WHAT == stamps ]]; then
  step in-kernel stamp diagnostic build
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -DWS_STAMPS -Icsrc tools/stamps/ws_stamps.hip csrc/device_window.cpp -o /tmp/ws_stamps \
    && timeout -k 10 120 /tmp/ws_stamps 4096 > "$OUT/ws_stamps.txt" 2>&1 && timeout -k 10 120 /tmp/ws_stamps 16384 >> "$OUT/ws_stamps.txt" 2>&1
  rc=$?; cat "$OUT/ws_stamps.txt"; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == rehearse ]]; then
  step "rank-0 render cost of an 8-GPU frame on one GPU (rehearsal, pipeline off / on)"
  for pl in 0 1; do
    timeout -k 10 300 python3 bench.py --rehearse-gpus 8 --pipeline $pl --json-out "$OUT/rehearse8_pipeline$pl.json" > "$OUT/rehearse8_pipeline$pl.log" 2>&1
    rc=$?; tail -1 "$OUT/rehearse8_pipeline$pl.log" | cut -c1-200; [[ $rc == 0 ]] || exit $rc
  done
  timeout -k 10 300 python3 bench.py --pipeline 1 --json-out "$OUT/bench_n1_pipeline1.json" > "$OUT/bench_n1_pipeline1.log" 2>&1
  rc=$?; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == handoff ]]; then
  step "sampler hand-off: spin vs futex, NUMA-pinned vs not (alternating, twice)"
  for rep in 1 2; do
    for cfg in "200 numa" "0 numa" "200 off" "0 off"; do
      set -- $cfg
      ROCMDASH_SAMPLER_SPIN_US=$1 ROCMDASH_PIN_SAMPLERS=$2 timeout -k 10 300 python3 bench.py \
        --json-out "$OUT/handoff_spin$1_$2_$rep.json" > "$OUT/handoff.log" 2>&1
      rc=$?; [[ $rc == 0 ]] || { tail -5 "$OUT/handoff.log"; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/handoff_spin$1_$2_$rep.json')); print('spin=$1 pin=$2', d['value'], d['ms_per_step'], d['p50_refresh_ms'], d['sampler_p50_us'], d['sampler_p99_us'], d['sampler_threads'])"
    done
  done
fi
if [[ $WHAT == cores ]]; then
  step "per-core sampler read cost"
  timeout -k 10 300 python3 tools/probes/probe_sampler_cores.py --out "$OUT/sampler_cores.json" > "$OUT/sampler_cores.log" 2>&1
  rc=$?; cat "$OUT/sampler_cores.log" | grep -v amdgpu.ids; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == envs ]]; then
  step "runtime knobs: polling signal waits, device-side kernel arguments (alternating, twice)"
  for rep in 1 2; do
    for cfg in "base" "HSA_ENABLE_INTERRUPT=0" "HIP_FORCE_DEV_KERNARG=1" "HSA_ENABLE_INTERRUPT=0 HIP_FORCE_DEV_KERNARG=1"; do
      tag=$(echo "$cfg" | tr ' =' '__')
      if [[ $cfg == base ]]; then envs=(); else read -r -a envs <<< "$cfg"; fi
      env "${envs[@]}" timeout -k 10 300 python3 bench.py --json-out "$OUT/envs_${tag}_$rep.json" > "$OUT/envs.log" 2>&1
      rc=$?; [[ $rc == 0 ]] || { tail -5 "$OUT/envs.log"; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/envs_${tag}_$rep.json')); print('$tag', d['value'], d['ms_per_step'], d['p50_refresh_ms'], d['p50_breakdown_ms'], d['sampler_p50_us'])"
    done
  done
fi
if [[ $WHAT == counterset ]]; then
  step "device-counting read cost per counter set"
  for set in ${COUNTER_SETS:-GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum SQ_VALU_MFMA_BUSY_CYCLES GRBM_COUNT,GRBM_GUI_ACTIVE \
             TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum GRBM_COUNT,GRBM_GUI_ACTIVE,SQ_VALU_MFMA_BUSY_CYCLES,TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum}; do
    timeout -k 10 120 python3 tools/probes/probe_counter_cost.py $set >> "$OUT/counter_cost.jsonl" 2> "$OUT/counter_cost.err"
    rc=$?; tail -1 "$OUT/counter_cost.jsonl"; [[ $rc == 0 ]] || { tail -5 "$OUT/counter_cost.err"; exit $rc; }
  done
fi
if [[ $WHAT == long ]]; then
  step "long-window statistics: GPU tests + micro-benchmark + kernel trace"
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_long_window.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_long.log" 2>&1
  rc=$?; tail -15 "$OUT/pytest_long.log"; [[ $rc == 0 ]] || exit $rc
  timeout -k 10 600 python3 tools/bench_long_window.py --out "$OUT/bench_long_window.json" > "$OUT/bench_long_window.log" 2>&1
  rc=$?; grep -v amdgpu.ids "$OUT/bench_long_window.log"; [[ $rc == 0 ]] || exit $rc
  rm -rf "$OUT/prof_long"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_long" -o run --output-format csv \
    -- python3 tools/bench_long_window.py --windows 1048576 --iters 20 > "$OUT/prof_long.log" 2>&1
  rc=$?; tail -2 "$OUT/prof_long.log"; [[ $rc == 0 ]] || exit $rc
  step "rocprofv3 PMC of the long-window passes: LDS histogram traffic and bank conflicts"
  rm -rf "$OUT/pmc_long"
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    -d "$OUT/pmc_long" -o pmc --output-format csv \
    -- python3 tools/bench_long_window.py --windows 1048576 --iters 5 > "$OUT/pmc_long.log" 2>&1
  rc=$?; tail -2 "$OUT/pmc_long.log"; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == record ]]; then
  step record live telemetry under a bf16 GEMM load for CPU replay tests
  timeout -k 10 180 python3 -m rocmdash.runtime.record --out "$OUT/mi355x_capture.npz" --seconds 8 --load > "$OUT/record.log" 2>&1
  rc=$?; tail -2 "$OUT/record.log"; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == asyncprobe ]]; then
  step "device-counter read: synchronous vs ASYNC (pipelined) reads"
  hipcc -O2 --offload-arch=gfx950 -o /tmp/probe_counter_async tools/probes/probe_counter_async.cpp -I/opt/rocm/include \
    -L/opt/rocm/lib -lrocprofiler-sdk -Wl,-rpath,/opt/rocm/lib 2>/dev/null \
    && timeout -k 10 90 /tmp/probe_counter_async 200 > "$OUT/probe_counter_async.txt" 2>&1
  rc=$?; grep -v "^W20\|^E20" "$OUT/probe_counter_async.txt"; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == layout ]]; then
  step "SMU metrics table layout: raw blob next to amd-smi's decoding"
  hipcc -O2 -o /tmp/probe_metrics_layout tools/probes/probe_metrics_layout.cpp -I/opt/rocm/include -L/opt/rocm/lib -lamd_smi \
    -Wl,-rpath,/opt/rocm/lib 2>/dev/null && timeout -k 10 60 /tmp/probe_metrics_layout > "$OUT/metrics_layout.txt" 2>&1
  rc=$?; head -40 "$OUT/metrics_layout.txt" | cut -c1-200; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == pcie ]]; then
  step "units of the SMU PCIe bandwidth figure against a pinned H2D stream"
  timeout -k 10 120 python3 tools/probes/probe_pcie_units.py > "$OUT/probe_pcie_units.txt" 2>&1
  rc=$?; grep -v amdgpu.ids "$OUT/probe_pcie_units.txt"; [[ $rc == 0 ]] || exit $rc
fi
if [[ $WHAT == nodewin ]]; then
  step "node-wide window statistics: GPU tests, bench with the extra all-gather + selection, kernel trace"
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "node_" > "$OUT/pytest_nodewin.log" 2>&1
  rc=$?; tail -6 "$OUT/pytest_nodewin.log"; [[ $rc == 0 ]] || exit $rc
  timeout -k 10 300 python3 bench.py --node-window --json-out "$OUT/bench_n1_nodewin.json" > "$OUT/bench_nodewin.log" 2>&1
  rc=$?; tail -1 "$OUT/bench_nodewin.log" | cut -c1-200; [[ $rc == 0 ]] || exit $rc
  rm -rf "$OUT/prof_nodewin"
  ROCMDASH_COUNTERS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_nodewin" -o run --output-format csv \
    -- python3 bench.py --node-window --steps 200 --warmup 20 > "$OUT/prof_nodewin.log" 2>&1
  rc=$?; tail -2 "$OUT/prof_nodewin.log"; [[ $rc == 0 ]] || exit $rc
fi
step done
