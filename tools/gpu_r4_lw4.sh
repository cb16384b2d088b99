#!/bin/bash
# Long-window pass 0: how the rings' workgroups share the chip. The service's 8 + 4 rings
# give 512 workgroups of 1 MB (8 series) and 512 of 0.5 MB (4 series) at W = 2^24: if a
# workgroup's stream is latency-bound, the 4-series workgroups finish at half time and
# the 8-series ones then run at half the chip's occupancy. Per-pass kernel times for the
# ring layouts 8+4, 8, 4, 12 and 4+4+4.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r4_lw4}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -m rocmdash._build --check || { echo "stale native build"; exit 3; }
for layout in 8+4 8 4 12 4+4+4; do
  tag=${layout//+/_}
  echo "== $(date +%T) layout $layout"
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$tag" -o run \
    -- python3 tools/bench_long_window.py --windows 16777216 --shapes telemetry,normal --iters 20 \
       --layout "$layout" > "$OUT/layout_$tag.log" 2>&1 || { tail -5 "$OUT/layout_$tag.log"; exit 1; }
  grep p50_us "$OUT/layout_$tag.log" | cut -c1-160
  f=$(find "$OUT/trace_$tag" -name "*kernel_trace.csv" | head -1 || true)
  [[ -n "$f" ]] && python3 tools/lw_trace_phases.py "$f" 10 > "$OUT/phases_$tag.txt" && cat "$OUT/phases_$tag.txt"
done
echo "== $(date +%T) done"
