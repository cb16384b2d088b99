#!/bin/bash
# One-off GPU probes of round 5 (one parameterised script instead of one file per lease):
#   tools/gpu_probe.sh hbm        known-traffic kernels under rocprofv3 --pmc (TCC request
#                                 sizes, DRAM vs fabric) + the HBM footprint stages
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
  *)
    echo "unknown probe $what" >&2
    exit 2
    ;;
esac
echo "probe $what done: $out"
