#!/bin/bash
# A/B of the world-size-1 host-out refresh (stats kernel writes pinned host memory) against
# the D2H copy, alternating twice on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for h in 1 0 1 0; do
  ROCMDASH_HOST_OUT=$h timeout -k 10 200 python3 bench.py --json-out gpurun_out/ab_hostout_$h.json > gpurun_out/ab_hostout.log 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_hostout_$h.json')); print('host_out=$h', d['value'], d['ms_per_step'], d['p50_refresh_ms'], d['p90_refresh_ms'], d['p50_breakdown_ms'], d['sampler_p50_us'])"
done
