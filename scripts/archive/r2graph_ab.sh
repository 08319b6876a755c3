#!/bin/bash
# Graph mode after releasing grads before the recording: GPU graph tests, then
# eager vs --graph 1 at ResNet-50 x256 (two interleaved rounds) and the
# reference's CIFAR shape (scripts/bench_cifar.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2gab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_graphs.log 2>&1 || { tail -30 $OUT/pytest_graphs.log; exit 1; }
tail -1 $OUT/pytest_graphs.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --cpu-baseline 0 --kernel-rates 0 --parity 0 > /dev/null 2> $OUT/compile.err || exit 1
for round in 1 2; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --graph $g --steps 30 --warmup 4 --cpu-baseline 0 --kernel-rates 0 --parity 0 > $OUT/r50_g${g}_$round.json 2> $OUT/r50_g${g}_$round.err || { tail -5 $OUT/r50_g${g}_$round.err; exit 1; }
    grep '^{' $OUT/r50_g${g}_$round.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'model': 'resnet50', 'batch': 256, 'graph': $g, 'round': $round, 'value': round(d['value'],1), 'ms_per_step': round(d['ms_per_step'],3)}))" | tee -a $OUT/summary.jsonl
  done
done
timeout -k 10 400 python -u scripts/bench_cifar.py --steps 50 > $OUT/cifar.jsonl 2> $OUT/cifar.err || { tail -5 $OUT/cifar.err; exit 1; }
cat $OUT/cifar.jsonl
