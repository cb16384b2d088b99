#!/bin/bash
# GPU-box A/B: the 1-GPU bench with the whole process started on the GPU's sysfs-local
# NUMA node vs the other node (taskset from exec; the sampler threads still pin
# themselves as configured), alternating.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
dev=$(readlink -f /sys/class/drm/card0/device)
node=$(cat "$dev/numa_node")
local_cpus=$(cat "$dev/local_cpulist")
remote=""
for n in /sys/devices/system/node/node*; do
  id=${n##*node}
  if [[ $id != "$node" ]]; then remote=$(cat "$n/cpulist"); break; fi
done
echo "numa_node $node local $local_cpus remote $remote"
for i in 1 2 3; do
  for side in local remote; do
    cpus=$local_cpus; [[ $side == remote ]] && cpus=$remote
    timeout -k 10 300 taskset -c "$cpus" python3 bench.py --json-out "$OUT/numa_bench_${side}_$i.json" > "$OUT/numa_bench_${side}_$i.log" 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('$OUT/numa_bench_${side}_$i.json')); print('$side', d['value'], d['ms_per_step'], d['p50_refresh_ms'], d['sampler_p50_us'])"
  done
done
