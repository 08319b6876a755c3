#!/bin/bash
# Reduction-grid sweep of the chunk-map engine (Σg², unpack+Σg²): grid cap x
# contiguous ranges vs grid-stride, R50 and R152x2 (bench_kernels rows).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r2d}
J=$OUT/${TAG}_red.jsonl
: > $J
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
for m in "resnet50 1" "resnet152 2"; do
  set -- $m
  for grid in ${GRIDS:-2048 8192 65536}; do
    for lib in ${LIBS:-default gred4}; do
      L=distributed_training_amd/lib/libgsync.so; [ $lib != default ] && L=distributed_training_amd/lib/variants/libgsync_$lib.so
      GSYNC_LIB=$L GS_RED_GRID=$grid timeout -k 10 300 python -u bench_kernels.py --model $1 --replicas $2 --skip-torch --iters 50 --tag g${grid}_$lib >> $J 2> $OUT/${TAG}_bk.err || { tail -20 $OUT/${TAG}_bk.err; exit 1; }
    done
  done
done
python3 - "$J" <<'PY'
import json,sys,collections
rows=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]
d=collections.defaultdict(list)
for r in rows:
    if 'sqnorm' in r['kernel']: d[(r['model'],r['kernel'],r['tag'])].append(r['GBps'])
for k in sorted(d): print(k, ' '.join(f'{x:7.0f}' for x in d[k]))
PY
