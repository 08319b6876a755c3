#!/bin/bash
# Small, launch-bound steps: libgsync DDP vs torch DDP on the same GPU (host overhead of the hook path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2w; mkdir -p $OUT
for m in "resnet18 8" "resnet18 32" "resnet50 16"; do
  set -- $m
  for impl in libgsync torch; do
    timeout -k 10 300 python -u bench.py --model $1 --batch $2 --impl $impl --cpu-baseline 0 --kernel-rates 0 --parity 0 --steps 30 --warmup 5 > $OUT/$1_$2_$impl.json 2> $OUT/$1_$2_$impl.err || { tail -5 $OUT/$1_$2_$impl.err; exit 1; }
    grep '^{' $OUT/$1_$2_$impl.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model': '$1', 'batch': $2, 'impl': '$impl', 'value': round(d['value'],1), 'ms_per_step': round(d['ms_per_step'],3)}))" | tee -a $OUT/summary.jsonl
  done
done
