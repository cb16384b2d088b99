#!/bin/bash
# GPU-box A/B: is the device-counter read's per-process cost (70 vs 140 us) set by the
# NUMA node the process starts on? Runs probe_counter_ctx pinned (taskset, from exec)
# to the GPU's local CPUs and to CPUs of another node, alternating.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
dev=$(readlink -f /sys/class/drm/card0/device)
node=$(cat "$dev/numa_node")
local_cpus=$(cat "$dev/local_cpulist")
echo "gpu $dev numa_node $node local_cpus $local_cpus"
for n in /sys/devices/system/node/node*; do echo "$(basename $n): $(cat $n/cpulist)"; done
remote=""
for n in /sys/devices/system/node/node*; do
  id=${n##*node}
  if [[ $id != "$node" ]]; then remote=$(cat "$n/cpulist"); break; fi
done
echo "remote cpus: $remote"
hipcc -O2 --offload-arch=gfx950 tools/probes/probe_counter_ctx.cpp -I/opt/rocm/include -L/opt/rocm/lib \
  -lrocprofiler-sdk -Wl,-rpath,/opt/rocm/lib -o "$OUT/pcc" || exit 1
for i in 1 2 3 4 5; do
  echo -n "local  "; timeout -k 10 60 taskset -c "$local_cpus" "$OUT/pcc" 300 2>/dev/null | grep "{" || exit 1
  if [[ -n $remote ]]; then echo -n "remote "; timeout -k 10 60 taskset -c "$remote" "$OUT/pcc" 300 2>/dev/null | grep "{" || exit 1; fi
done
