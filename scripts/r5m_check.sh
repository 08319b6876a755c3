#!/bin/bash
# Round 5: the producer-side tail without its pk0 packet (level 2): the DDP GPU
# tests, then two default bench runs (legs off) for the tail split; then Σg² on
# three layouts of the same elements (scripts/sqnorm_shapes.py).  The clip / ZeRO
# GPU tests ride along: gs_sqnorm_partial_out now zeroes the buffer past its count.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_native_hook.py tests/test_clip_fold.py tests/test_zero_ds_step.py tests/test_gpu_zero.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_ddp.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_ddp.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="" scripts/variant_rows.sh $OUT
timeout -k 10 120 python -u scripts/sqnorm_shapes.py > $OUT/sqnorm_shapes.jsonl 2> $OUT/sqnorm_shapes.err || { tail -20 $OUT/sqnorm_shapes.err; exit 1; }
cat $OUT/sqnorm_shapes.jsonl
