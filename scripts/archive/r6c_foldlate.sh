#!/bin/bash
# Round 6: the folded clip's coefficient formed after each workgroup's first loads
# (GS_FOLD_LATE=1, a library variant in lib/variants/foldlate/) — first its bit-exactness
# (the clip-fold, ZeRO-step and kernel tests on the variant), then interleaved with the
# default over two rounds (scripts/variant_rows.sh): the clip-path rows, configs[3]'s
# N=8-shard clip path, the tail.  The variant was built on the CPU beforehand
# (make -C distributed_training_amd/csrc OUTDIR=../lib/variants/foldlate
#  OBJDIR=../../build/gsync_foldlate EXTRA_DEFS=-DGS_FOLD_LATE=1); the option was
# removed after this A/B lost (profiles/r6/r6c_foldlate_rows.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6c; mkdir -p $OUT
export TMPDIR=/tmp
GSYNC_LIB=$PWD/distributed_training_amd/lib/variants/foldlate/libgsync.so timeout -k 10 600 python -u -m pytest \
  tests/test_clip_fold.py tests/test_zero_ds_step.py tests/test_gpu_kernels.py tests/test_gpu_clip_fused.py \
  tests/test_fused_norm_amp.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_foldlate.log 2>&1
rc=$?; tail -3 $OUT/pytest_foldlate.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="foldlate" scripts/variant_rows.sh $OUT
