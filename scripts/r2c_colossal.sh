#!/bin/bash
# BASELINE configs[4] at full size through the Colossal Booster shim
# (TorchDDPPlugin + fp16 + HybridAdam, libgsync DDP underneath) beside the same
# step on torch alone (torch DDP + GradScaler + fused AdamW), one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2c; mkdir -p $OUT
for m in "resnet152 128" "resnet50 256"; do
  set -- $m
  for impl in libgsync torch; do
    extra=""; [ $impl = libgsync ] && extra="--parity 1"
    timeout -k 10 400 python -u bench.py --engine colossal --model $1 --batch $2 --impl $impl --cpu-baseline 0 --kernel-rates 0 $extra > $OUT/colossal_$1_$2_$impl.json 2> $OUT/colossal_$1_$2_$impl.err || { tail -5 $OUT/colossal_$1_$2_$impl.err; exit 1; }
    grep '^{' $OUT/colossal_$1_$2_$impl.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d.get('parity') or {}; r=d.get('roofline') or {}
print(json.dumps({'engine': 'colossal', 'model': '$1', 'batch': $2, 'impl': '$impl', 'value': round(d['value'],1), 'ms_per_step': round(d['ms_per_step'],3), 'parity_ok': p.get('ok'), 'update_frac': r.get('frac'), 'update_ms': r.get('avg_launch_ms')}))" | tee -a $OUT/summary.jsonl
  done
done
