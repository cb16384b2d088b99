#!/bin/bash
set -u
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/probes
mkdir -p "$OUT"; cd "$(dirname "$0")"
hipcc -O2 --offload-arch=gfx950 -o "$OUT/probe_devcount" probe_devcount.cpp -I/opt/rocm/include -L/opt/rocm/lib -lrocprofiler-sdk -Wl,-rpath,/opt/rocm/lib 2>/dev/null
timeout -k 5 180 "$OUT/probe_devcount" > "$OUT/probe_devcount2.txt" 2>&1; echo rc=$?
cat "$OUT/probe_devcount2.txt"
