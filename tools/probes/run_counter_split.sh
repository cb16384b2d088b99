#!/bin/bash
# GPU-box run of probe_counter_split: the device-counter set split over several
# concurrently running contexts, started from the GPU's local NUMA node and from a
# remote one (the read cost depends on the node the runtime started on, placement.py).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p "$OUT"
dev=$(readlink -f /sys/class/drm/card0/device)
node=$(cat "$dev/numa_node")
local_cpus=$(cat "$dev/local_cpulist")
remote=""
for n in /sys/devices/system/node/node*; do
  id=${n##*node}
  if [[ $id != "$node" ]]; then remote=$(cat "$n/cpulist"); break; fi
done
echo "gpu numa_node $node local $local_cpus remote $remote"
hipcc -O2 --offload-arch=gfx950 tools/probes/probe_counter_split.cpp -I/opt/rocm/include -L/opt/rocm/lib \
  -lrocprofiler-sdk -Wl,-rpath,/opt/rocm/lib -o "$OUT/pcs" || exit 1
for i in 1 2; do
  for where in local remote; do
    cpus=$local_cpus; [[ $where == remote ]] && cpus=$remote
    [[ -n $cpus ]] || continue
    echo "== $where run $i"
    timeout -k 10 90 taskset -c "$cpus" "$OUT/pcs" 300 2> "$OUT/pcs.err" | grep "{" || { tail -5 "$OUT/pcs.err"; exit 1; }
  done
done
