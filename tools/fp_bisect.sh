set -o pipefail
O=gpurun_out/r3fp; mkdir -p $O
timeout -k 10 120 python tools/footprint_probe.py --world 1 --seconds 8 --out $O/fp_live.json > $O/fp_live.log 2>&1 &&
HSA_ENABLE_INTERRUPT=1 timeout -k 10 120 python tools/footprint_probe.py --world 1 --seconds 8 --out $O/fp_live_int1.json > $O/fp_live_int1.log 2>&1 &&
ROCMDASH_COUNTER_HZ=10 timeout -k 10 120 python tools/footprint_probe.py --world 1 --seconds 8 --out $O/fp_live_ctr10.json > $O/fp_live_ctr10.log 2>&1
cat $O/fp_live*.json | cut -c1-1500; env | grep -i "HSA_\|HIP_\|ROC" | sort
