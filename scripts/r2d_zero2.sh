#!/bin/bash
# BASELINE configs[3] (DeepSpeed-style ZeRO-2, ResNet-50 bf16, AdamW, clip 1.0) on one GPU:
# libgsync ZeroDataParallel vs torch FSDP(SHARD_GRAD_OP) with bf16 mixed precision + fused AdamW.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2d; mkdir -p $OUT
for impl in libgsync torch; do
  extra=""; [ $impl = libgsync ] && extra="--parity 1"
  timeout -k 10 400 python -u bench.py --engine zero2 --optimizer adam --model resnet50 --batch 256 --impl $impl --cpu-baseline 0 --kernel-rates 0 $extra > $OUT/zero2_$impl.json 2> $OUT/zero2_$impl.err || { tail -8 $OUT/zero2_$impl.err; exit 1; }
  grep '^{' $OUT/zero2_$impl.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d.get('parity') or {}; r=d.get('roofline') or {}
print(json.dumps({'engine': 'zero2', 'model': 'resnet50', 'batch': 256, 'impl': '$impl', 'value': round(d['value'],1), 'ms_per_step': round(d['ms_per_step'],3), 'parity_ok': p.get('ok'), 'update_frac': r.get('frac'), 'update_ms': r.get('avg_launch_ms'), 'zero_step_window_ms': d.get('zero_step_window_ms')}))" | tee -a $OUT/summary.jsonl
done
