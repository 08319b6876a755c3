#!/bin/bash
# Headline-size steps: libgsync DDP vs torch DDP on the same GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2x; mkdir -p $OUT
for m in "resnet50 256 sgd" "resnet50 256 adam" "resnet152 128 sgd"; do
  set -- $m
  for impl in libgsync torch; do
    timeout -k 10 400 python -u bench.py --model $1 --batch $2 --optimizer $3 --impl $impl --cpu-baseline 0 --kernel-rates 0 --parity 0 > $OUT/$1_$2_$3_$impl.json 2> $OUT/$1_$2_$3_$impl.err || { tail -5 $OUT/$1_$2_$3_$impl.err; exit 1; }
    grep '^{' $OUT/$1_$2_$3_$impl.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model': '$1', 'batch': $2, 'optimizer': '$3', 'impl': '$impl', 'value': round(d['value'],1), 'ms_per_step': round(d['ms_per_step'],3)}))" | tee -a $OUT/summary.jsonl
  done
done
