#!/bin/bash
# Round 5: balanced reduction grids (GS_RED_BALANCED: every workgroup of a capped
# reduction grid strides over the same number of chunk groups), alone, with
# groups of 4 chunks, with a 4 Ki fused grid, and with the one-level fused fold
# (GS_RED_ONE_LEVEL) — library variants in
# lib/variants/<name>/ interleaved with the default over two rounds (the
# kernel rates, the N=8-shard clip path, the exposed tail).  One JSON line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5i; mkdir -p $OUT
export TMPDIR=/tmp
# the one-level fold's numerics first: the reduction / clip GPU tests on that library
GSYNC_LIB=$PWD/distributed_training_amd/lib/variants/onelevel/libgsync.so timeout -k 10 400 python -u -m pytest tests/test_clip_fold.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_onelevel.log 2>&1
rc=$?; tail -3 $OUT/pytest_onelevel.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS:-redbal redbal_g4 redbal_fg4k onelevel}" scripts/variant_rows.sh $OUT
