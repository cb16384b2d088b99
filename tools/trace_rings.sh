set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/trace16; mkdir -p $OUT
for cfg in "r16|11 5" "r11|11"; do
  name=${cfg%%|*}; rings=${cfg#*|}
  rm -rf $OUT/$name
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 tools/bench_kernel.py --iters 600 --windows 4096 --rings $rings --ks 1 --signal 2 > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  python3 tools/summarize_prof.py "$(find $OUT/$name -name '*kernel_trace.csv' | head -1)" --out $OUT/$name.json > /dev/null || exit 1
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))['kernels']
for k,v in d.items():
    if 'window_stats_kernel' in k: print(sys.argv[2], k[:45], v['dispatches'], 'grid', v['Grid_Size_X'], 'p10/p50/p90', v['p10_us'], v['p50_us'], v['p90_us'])
" $OUT/$name.json "$name"
  grep '"k_new": 1' $OUT/$name.log | cut -c1-200
done
