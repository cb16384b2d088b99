#!/bin/bash
# GPU-box capability probe (amd-smi, rocprofiler-sdk device counting, torch, RCCL availability).
set -u
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/probes
mkdir -p "$OUT"
cd "$(dirname "$0")"
hipcc -O2 -o "$OUT/probe_amdsmi" probe_amdsmi.cpp -I/opt/rocm/include -L/opt/rocm/lib -lamd_smi -Wl,-rpath,/opt/rocm/lib 2>/dev/null
hipcc -O2 --offload-arch=gfx950 -o "$OUT/probe_devcount" probe_devcount.cpp -I/opt/rocm/include -L/opt/rocm/lib -lrocprofiler-sdk -Wl,-rpath,/opt/rocm/lib 2>/dev/null
echo "== id"; id; echo "== nproc $(nproc)"
echo "== amd-smi cli"; timeout -k 5 60 amd-smi static --asic --board 2>&1 | head -60 > "$OUT/amdsmi_static.txt"; head -40 "$OUT/amdsmi_static.txt"
echo "== probe_amdsmi"; timeout -k 5 120 "$OUT/probe_amdsmi" 2>&1 | tee "$OUT/probe_amdsmi.txt"
echo "== probe_devcount"; timeout -k 5 120 "$OUT/probe_devcount" 2>&1 | tee "$OUT/probe_devcount.txt"
echo "== torch"; timeout -k 5 300 python -c "
import torch, torch.distributed as dist
print(torch.__version__, torch.cuda.is_available(), torch.cuda.device_count())
p=torch.cuda.get_device_properties(0); print(p.name, p.gcnArchName, p.multi_processor_count, p.total_memory/2**30)
print('nccl', dist.is_nccl_available(), torch.cuda.nccl.version())
" 2>&1 | tee "$OUT/torch.txt"
ls /sys/class/drm/ | head; cat /sys/class/drm/card*/device/gpu_metrics 2>/dev/null | wc -c
ls -la /dev/kfd /dev/dri 2>&1 | head
