#!/bin/bash
# Kernel-trace A/B of the headline bench across built trees (rocprofv3, device counters
# off under the profiler), alternating. Usage: bash tools/ab_tree_prof.sh REPS DIR1 DIR2 ...
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abprof; mkdir -p "$OUT"
export TMPDIR=/tmp
REPS=$1; shift
for rep in $(seq "$REPS"); do
  for dir in "$@"; do
    tag=$(basename "$dir"); [[ $dir == . ]] && tag=head
    rm -rf "$OUT/${tag}_$rep"
    (cd "$dir" && ROCMDASH_COUNTERS=0 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d "$OLDPWD/$OUT/${tag}_$rep" -o run \
      --output-format csv -- python3 bench.py --steps 1000 --warmup 20 --timing-steps 0 --json-out "$OLDPWD/$OUT/${tag}_$rep.json") \
      > "$OUT/${tag}_$rep.log" 2>&1 || { tail -5 "$OUT/${tag}_$rep.log"; exit 1; }
    python3 - "$OUT/${tag}_$rep" "$tag" "$OUT/${tag}_$rep.json" <<'PY'
import csv, glob, json, statistics, sys
f = glob.glob(sys.argv[1] + "/*kernel_trace.csv")[0]
rows = [r for r in csv.DictReader(open(f)) if "window_stats_kernel<" in r["Kernel_Name"]]
name = max({r["Kernel_Name"] for r in rows}, key=lambda n: sum(r["Kernel_Name"] == n for r in rows))  # the steady-state launch
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if r["Kernel_Name"] == name]
b = json.load(open(sys.argv[3]))
print(sys.argv[2], name.split("(")[0].split("::")[-1], "p50 %.2f p10 %.2f n=%d" % (statistics.median(d), sorted(d)[len(d) // 10], len(d)),
      "| bench p50 %.4f ms, device+gather %.4f ms" % (b["p50_refresh_ms"], b["p50_breakdown_ms"]["device+gather"]))
PY
  done
done
