export TMPDIR=/tmp; mkdir -p gpurun_out/lwt
for arm in old new; do dir=.; [[ $arm == old ]] && dir=ab_old
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lwt/$arm -o run --output-format csv -- python3 $dir/tools/bench_long_window.py --windows 16777216 --shapes normal --iters 20 > gpurun_out/lwt/$arm.log 2>&1 || exit 1
done
