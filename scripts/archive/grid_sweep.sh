#!/bin/bash
# Grid-cap x task-size x ILP sweep (scripts/copy_micro.hip found one-shot
# workgroups beat a resident looping grid by ~20 % at HBM sizes).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for lib in libgsync variants/libgsync_ilp1; do
  for grid in 2048 65536; do
    for MR in resnet50:1 resnet152:2; do
      GSYNC_LIB=distributed_training_amd/lib/$lib.so GS_MAX_GRID=$grid timeout -k 10 200 python -u scripts/sweep_tasks.py \
        --model ${MR%%:*} --replicas ${MR#*:} --tasks ${TASKS:-0,256,512,1024} --rounds 3 --ops pack,unpack,sgd,adam \
        --tag "$(basename $lib)_g$grid" >> $OUT/grid_sweep.jsonl 2>> $OUT/grid_sweep.err || exit 1
    done
  done
done
