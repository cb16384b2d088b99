#!/bin/bash
# A/B on one MI355X box: closed-loop sampling (one prefetched read per source per refresh)
# vs free-running sources (each refresh waits for >= 1 new row per source), 3 alternating
# rounds of the N = 1 headline bench. Usage (via gpurun): bash tools/ab_sampling.sh [outdir]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r3sampling}; mkdir -p $O
python3 -m rocmdash._build --check || exit 3
for i in 1 2 3; do
  for m in closed free; do
    echo "[ab_sampling] $(date +%T) round $i $m"
    timeout -k 10 200 python bench.py --steps 4000 --warmup 100 --e2e-s 0 --timing-steps 0 --sampling $m \
        > $O/bench_$m\_$i.json 2> $O/bench_$m\_$i.err || exit 1
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["p50_refresh_ms"], d["p90_refresh_ms"], d["ms_per_step"], d["sampler_p50_us"],
          d["sampler_mean_us"], d["p50_breakdown_ms"], d["hardware_reads_per_s"])
PY
