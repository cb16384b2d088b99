#!/bin/bash
# A/B on one box: where the counter sampler thread and the runtime's busy-polling thread
# run (rocmdash/runtime/threads.py, agent.py pin_samplers), alternating 3 rounds:
#   numa   samplers on the GPU-local NUMA node (default)
#   init   samplers on the node the runtime was started on (the calibrated fast node)
#   spin   samplers GPU-local + the poller moved there too
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r3pin}; mkdir -p $O
for i in 1 2 3; do
  for v in numa init spin; do
    echo "[ab_pin] $(date +%T) round $i $v"
    case $v in
      numa) env_="ROCMDASH_PIN_SAMPLERS=numa";;
      init) env_="ROCMDASH_PIN_SAMPLERS=init";;
      spin) env_="ROCMDASH_PIN_SAMPLERS=numa ROCMDASH_PIN_SPINNER=1";;
    esac
    env $env_ timeout -k 10 200 python bench.py --steps 3000 --warmup 100 --e2e-s 0 --timing-steps 0 \
        > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit 1
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["p50_refresh_ms"], d["ms_per_step"], d["sampler_p50_us"], d["init_placement"]["node"] if d["init_placement"] else None, d["sampler_threads"], d["sched_idle_threads"])
PY
