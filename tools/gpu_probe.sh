#!/bin/bash
# One-off GPU probes of round 5 (one parameterised script instead of one file per lease):
#   tools/gpu_probe.sh hbm        known-traffic kernels under rocprofv3 --pmc (TCC request
#                                 sizes, DRAM vs fabric) + the HBM footprint stages
#   tools/gpu_probe.sh footprint  the HBM footprint stages only (fresh process per stage)
#   tools/gpu_probe.sh hipenv     a HIP process's first kernel / extra streams under runtime knobs
#   tools/gpu_probe.sh nodecpu    node-total CPU of the supervised service at production
#                                 rates: 8 oversubscribed ranks + the node counter process,
#                                 and 1 rank with / without it
# Results land in gpurun_out/<name>/ (copy what is judged into profiles/).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
what=${1:?usage: gpu_probe.sh hbm}
out="$R/gpurun_out/probe_$what"
mkdir -p "$out" build/probes
export TMPDIR=/tmp

case "$what" in
  hbm)
    hipcc -O3 --offload-arch=gfx950 -o build/probes/probe_hbm_bytes tools/probes/probe_hbm_bytes.hip 2>/dev/null
    hipcc -O3 --offload-arch=gfx950 -o build/probes/probe_hip_init tools/probes/probe_hip_init.hip 2>/dev/null
    timeout -k 10 120 build/probes/probe_hbm_bytes 3 > "$out/plain.jsonl"
    i=0
    for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_32B_sum" \
               "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_GMI_32B_sum" \
               "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_DRAM_sum"; do
      i=$((i + 1))
      (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$out/pmc$i" -o run \
         -- "$R/build/probes/probe_hbm_bytes" 2) > "$out/pmc$i.log" 2>&1
    done
    timeout -k 10 400 python tools/probes/probe_hbm_footprint.py --hip-probe build/probes/probe_hip_init \
      > "$out/footprint.jsonl" 2> "$out/footprint.err"
    ;;
  footprint)
    hipcc -O3 --offload-arch=gfx950 -o build/probes/probe_hip_init tools/probes/probe_hip_init.hip 2>/dev/null
    timeout -k 10 400 python tools/probes/probe_hbm_footprint.py --hip-probe build/probes/probe_hip_init \
      > "$out/footprint.jsonl" 2> "$out/footprint.err"
    ;;
  hipenv)
    # what a HIP process's first kernel and each extra stream take, under runtime knobs
    hipcc -O3 --offload-arch=gfx950 -o build/probes/probe_hip_init tools/probes/probe_hip_init.hip 2>/dev/null
    bdf_path=$(python3 -c "from rocmdash.runtime.topology import bdf_of_hip_device; from rocmdash.runtime.agent import bdf_path; print(bdf_path(bdf_of_hip_device(0)) + '/mem_info_vram_used')")
    : > "$out/hipenv.jsonl"
    for envs in "" "GPU_MAX_HW_QUEUES=1" "HSA_SCRATCH_SINGLE_LIMIT=1048576" "HSA_SCRATCH_MEM=1048576" \
                "HIP_INITIAL_DM_SIZE=0" "HSA_DISABLE_FRAGMENT_ALLOCATOR=1" "ROC_AQL_QUEUE_SIZE=1024" \
                "GPU_STAGING_BUFFER_SIZE=1 GPU_XFER_BUFFER_SIZE=1" "HSA_NO_SCRATCH_RECLAIM=1" \
                "GPU_MAX_HW_QUEUES=1 HSA_SCRATCH_SINGLE_LIMIT=1048576"; do
      sleep 2  # the previous process's memory is freed asynchronously
      line=$(env $envs timeout -k 10 60 build/probes/probe_hip_init "$bdf_path" || echo '{"rc": "failed"}')
      echo "{\"env\": \"$envs\", \"r\": $line}" >> "$out/hipenv.jsonl"
    done
    cat "$out/hipenv.jsonl"
    ;;
  nodecpu)
    ROCMDASH_OVERSUBSCRIBE=1 timeout -k 10 400 python tools/node_cpu_probe.py --nproc 8 --counter-daemon on \
      --out "$out/node8_daemon.json" > "$out/node8_daemon.log" 2>&1
    timeout -k 10 300 python tools/node_cpu_probe.py --nproc 1 --counter-daemon on --out "$out/node1_daemon.json" \
      > "$out/node1_daemon.log" 2>&1
    timeout -k 10 300 python tools/node_cpu_probe.py --nproc 1 --counter-daemon off --out "$out/node1_own.json" \
      > "$out/node1_own.log" 2>&1
    ;;
  *)
    echo "unknown probe $what" >&2
    exit 2
    ;;
esac
echo "probe $what done: $out"
