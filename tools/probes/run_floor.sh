#!/bin/bash
# Kernel-trace floor probe + window-stats trace: this tree vs .ab_old/ (tools/ab_kernel.sh).
# (The uncached-buffer side of profiles/r02/onerow/ ran with a switch since removed.)
# Usage (via gpurun): bash tools/probes/run_floor.sh
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 tools/probes/probe_kernel_floor.hip -o /tmp/floor || exit 3
rm -rf "$OUT/floor"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/floor" -o floor --output-format csv -- /tmp/floor > "$OUT/floor.log" 2>&1 || exit $?
for rep in 1 2; do
  for side in new old; do
    dir=.; [[ $side == old ]] && dir=.ab_old
    rm -rf "$OUT/kt_${side}_$rep"
    (cd "$dir" && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OLDPWD/$OUT/kt_${side}_$rep" -o kt --output-format csv \
      -- python3 tools/bench_kernel.py --iters 300 --windows 4096 16384 --series 15 --ks 1 10) > "$OUT/kt_${side}_$rep.log" 2>&1 || exit $?
  done
done
echo "== done"
