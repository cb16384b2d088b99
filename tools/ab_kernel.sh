#!/bin/bash
# A/B of the window-stats kernel: this tree vs the build in .ab_old/ (an older tree,
# built in place), alternating, plus an LDS PMC pass of this tree's kernel.
# Usage (via gpurun, from the repo root): bash tools/ab_kernel.sh [reps]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
REPS=${1:-2}
ARGS="${AB_ARGS:---windows 4096 16384 --series 15 64 --ks 1 10 100 --iters 300}"
: > "$OUT/ab_kernel.jsonl"
for rep in $(seq "$REPS"); do
  for side in new old; do
    dir=.; [[ $side == old ]] && dir=.ab_old
    (cd "$dir" && timeout -k 10 300 python3 tools/bench_kernel.py $ARGS --out "/tmp/bk_$side.json") > "$OUT/ab_kernel_$side.log" 2>&1
    rc=$?; [[ $rc == 0 ]] || { tail -5 "$OUT/ab_kernel_$side.log"; exit $rc; }
    python3 -c "
import json
for r in json.load(open('/tmp/bk_$side.json')):
    r.update(side='$side', rep=$rep); print(json.dumps(r))" >> "$OUT/ab_kernel.jsonl"
  done
done
python3 - "$OUT/ab_kernel.jsonl" <<'EOF'
import json, sys, statistics
rows = [json.loads(l) for l in open(sys.argv[1])]
keys = sorted({(r["W"], r["series"], r["k_new"] or 0, r["path"]) for r in rows})
for k in keys:
    v = {s: [r["p50_us"] for r in rows if (r["W"], r["series"], r["k_new"] or 0, r["path"]) == k and r["side"] == s]
         for s in ("new", "old")}
    print(k, "new", v["new"], "old", v["old"])
EOF
rm -rf "$OUT/pmc_ab"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS \
  -d "$OUT/pmc_ab" -o pmc --output-format csv \
  -- python3 tools/bench_kernel.py --iters 40 --windows 4096 --series 15 --ks 1 > "$OUT/pmc_ab.log" 2>&1
rc=$?; tail -2 "$OUT/pmc_ab.log"; [[ $rc == 0 ]] || exit $rc
rm -rf "$OUT/pmc_ab_old"
(cd .ab_old && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS \
  -d "../$OUT/pmc_ab_old" -o pmc --output-format csv \
  -- python3 tools/bench_kernel.py --iters 40 --windows 4096 --series 15 --ks 1) > "$OUT/pmc_ab_old.log" 2>&1
rc=$?; tail -2 "$OUT/pmc_ab_old.log"; [[ $rc == 0 ]] || exit $rc
echo "== done"
