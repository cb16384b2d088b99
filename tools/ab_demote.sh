#!/bin/bash
# A/B on one box: the node service's SCHED_IDLE demotion of the runtime's busy-polling
# thread (rocmdash/runtime/threads.py) in the headline bench, alternating, plus the
# service footprint at production rates with the demotion.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r3demote}; mkdir -p $O
timeout -k 10 200 python tools/footprint_probe.py --world 1 --seconds 8 --out $O/footprint_w1.json > $O/footprint_w1.log 2>&1 &&
for i in 1 2; do
  for d in 0 1; do
    echo "[ab_demote] $(date +%T) run $i demote=$d"
    timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --e2e-s 0 --timing-steps 0 --demote-spin $d \
        > $O/bench_d${d}_$i.json 2> $O/bench_d${d}_$i.err || exit 1
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_d*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["p50_refresh_ms"], d["ms_per_step"], d["sampler_p50_us"], d["sched_idle_threads"])
PY
cat $O/footprint_w1.json
