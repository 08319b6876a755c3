#!/bin/bash
# Time every libgsync build variant under distributed_training_amd/lib/variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for lib in distributed_training_amd/lib/libgsync.so distributed_training_amd/lib/variants/*.so; do
  name=$(basename $lib .so)
  for m in "resnet50 1" "resnet152 2"; do
    set -- $m
    echo "== $name $1 x$2" | tee -a $OUT/kvariants.log
    GSYNC_LIB=$lib timeout -k 10 200 python -u bench_kernels.py --model $1 --replicas $2 --skip-torch --iters 30 | sed "s/^/$name /" >> $OUT/kvariants.log 2>> $OUT/kvariants.err || exit 1
  done
done
