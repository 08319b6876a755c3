#!/bin/bash
# Round 5: the clip / reduction GPU tests on the wave-0 clip fold, then the raw
# Σg² partials' workgroup cap (GS_RAW_WORKGROUPS 256 / 512 default / 1024 / 2048,
# library variants in lib/variants/<name>/) interleaved over two rounds:
# configs[3]'s N=8-shard clip path both forms, the exposed tail's split (level-2
# marks: start packets, kernel-carried stops).  One JSON line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_clip_fold.py tests/test_zero_ds_step.py tests/test_gpu_kernels.py tests/test_fused_norm_amp.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_subset.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu_subset.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS:-rawwg256 rawwg1024 rawwg2048}" scripts/variant_rows.sh $OUT
