#!/bin/bash
# copy ceiling + R50/R152 pack/unpack sweep for each build variant
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for lib in distributed_training_amd/lib/libgsync.so distributed_training_amd/lib/variants/*.so; do
  tag=$(basename $lib .so)
  GSYNC_LIB=$lib timeout -k 10 200 python -u scripts/copy_ceiling.py | sed "s/^{/{\"tag\": \"$tag\", /" >> $OUT/pack_ceiling.jsonl || exit 1
  for MR in resnet50:1 resnet152:2; do
    GSYNC_LIB=$lib timeout -k 10 150 python -u scripts/sweep_tasks.py --model ${MR%%:*} --replicas ${MR#*:} --tasks 0 --rounds 10 \
      --ops pack,unpack,sgd --tag $tag >> $OUT/pack_sweep.jsonl 2>> $OUT/pack_sweep.err || exit 1
  done
done
