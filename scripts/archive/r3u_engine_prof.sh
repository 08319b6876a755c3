#!/bin/bash
# rocprofv3 kernel stats of the ZeRO-2 (configs[3]) and Colossal ResNet-152 (configs[4]) bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=r3u; mkdir -p $OUT
for cfg in "zero2 resnet50 256 adam" "colossal resnet152 128 adam"; do
  set -- $cfg
  d=$OUT/prof_${TAG}_$1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $d -o bench -- python3 -u bench.py --engine $1 --model $2 --batch $3 --optimizer $4 --steps 10 --warmup 3 --cpu-baseline 0 --kernel-rates 0 --parity 0 > $OUT/${TAG}_bench_$1.json 2> $OUT/${TAG}_bench_$1.err || { tail -5 $OUT/${TAG}_bench_$1.err; exit 1; }
  s=$(find $d -name "*kernel_stats.csv" | head -1); cp "$s" $OUT/${TAG}_$1_kernel_stats.csv; rm -rf $d
  python3 -c "
import json; d=json.loads(open('$OUT/${TAG}_bench_$1.json').read().strip().splitlines()[-1])
print('$1', round(d['value'],1), round(d['roofline']['frac'],3), d['roofline']['avg_launch_ms'])"
done
