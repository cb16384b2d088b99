#!/bin/bash
# Phase stamps of the window-stats kernel, this tree vs .ab_old/ (see tools/ab_kernel.sh).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out; mkdir -p "$OUT"
for side in new old; do
  dir=.; [[ $side == old ]] && dir=.ab_old
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -DWS_STAMPS -I$dir/csrc $dir/tools/stamps/ws_stamps.hip $dir/csrc/device_window.cpp \
    -o /tmp/ws_stamps_$side || exit 3
done
: > "$OUT/ws_stamps_ab.txt"
for rep in 1 2; do
  for side in new old; do
    for W in 4096 16384; do
      echo "[$side rep $rep]" >> "$OUT/ws_stamps_ab.txt"
      timeout -k 10 120 /tmp/ws_stamps_$side $W 15 >> "$OUT/ws_stamps_ab.txt" 2>&1 || exit $?
    done
  done
done
cat "$OUT/ws_stamps_ab.txt"
