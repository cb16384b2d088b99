#!/bin/bash
# GPU-box A/B: device-counter read cost with ROCr's interrupt-driven signal waits
# (default) vs polling (HSA_ENABLE_INTERRUPT=0), alternating fresh processes.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PROBE_QUICK=1
for i in 1 2 3 4 5 6 7; do
  timeout -k 10 60 python3 -u tools/probes/probe_overlap.py 2>/dev/null | grep "{" || exit 1
  HSA_ENABLE_INTERRUPT=0 timeout -k 10 60 python3 -u tools/probes/probe_overlap.py 2>/dev/null | grep "{" || exit 1
done
