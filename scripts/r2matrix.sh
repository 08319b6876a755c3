#!/bin/bash
# Consolidated end-of-round matrix on one box: every engine / option of bench.py
# at full size, libgsync and the torch-only comparison where one exists.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2matrix; mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 4 --cpu-baseline 0 --kernel-rates 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; return 1; }
  grep '^{' $OUT/$name.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d.get('parity') or {}; r=d.get('roofline') or {}
print(json.dumps({'name': '$name', 'args': '$*', 'value': round(d['value'],1), 'ms_per_step': round(d['ms_per_step'],3), 'dtype': d['dtype'], 'parity_ok': p.get('ok'), 'update_frac': None if not r else round(r['frac'],3), 'tail_us': round(((d.get('grad_sync') or {}).get('tail_ms') or {}).get('total_timed_step', 0)*1e3,1)}))" | tee -a $OUT/summary.jsonl
}
run ddp_sgd_r50 || exit 1
run torch_sgd_r50 --impl torch --parity 0 || exit 1
run ddp_adam_r50 --optimizer adam || exit 1
run torch_adam_r50 --optimizer adam --impl torch --parity 0 || exit 1
run ddp_sgd_r50_bf16buckets --bucket-dtype bf16 || exit 1
run ddp_sgd_r50_overlap --optimizer-overlap 1 || exit 1
run ddp_sgd_r50_view --grad-as-bucket-view || exit 1
run ddp_sgd_r50_graph --graph 1 --parity 0 || exit 1
run zero1_adamw_r50 --engine zero1 --optimizer adam || exit 1
run zero2_adamw_r50 --engine zero2 --optimizer adam || exit 1
run torch_fsdp_zero2_r50 --engine zero2 --optimizer adam --impl torch --parity 0 || exit 1
run colossal_r152 --engine colossal --model resnet152 --batch 128 || exit 1
run torch_colossal_r152 --engine colossal --model resnet152 --batch 128 --impl torch --parity 0 || exit 1
run ddp_sgd_r152 --model resnet152 --batch 128 || exit 1
run torch_sgd_r152 --model resnet152 --batch 128 --impl torch --parity 0 || exit 1
echo "== done"
