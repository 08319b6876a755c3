#!/bin/bash
# Time libgsync build variants (interleaved, REPEAT rounds) with bench_kernels.py
#   VARIANTS="libgsync variants/libgsync_v_old ..." (relative to distributed_training_amd/lib)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
VARIANTS=${VARIANTS:-"libgsync $(cd distributed_training_amd/lib && ls variants/*.so | sed 's/\.so$//' | tr '\n' ' ')"}
for r in $(seq 1 ${REPEAT:-1}); do
for v in $VARIANTS; do
  lib=distributed_training_amd/lib/$v.so
  name=$(basename $v)
  MODELS=${MODELS:-resnet50:1 resnet152:2}
  for m in $MODELS; do
    mm=${m%%:*}; rep=${m#*:}
    echo "== $name $mm x$rep round $r" | tee -a $OUT/kvariants.log
    GSYNC_LIB=$lib timeout -k 10 200 python -u bench_kernels.py --model $mm --replicas $rep --skip-torch --iters 30 | sed "s/^/$name /" >> $OUT/kvariants.log 2>> $OUT/kvariants.err || exit 1
  done
done
done
