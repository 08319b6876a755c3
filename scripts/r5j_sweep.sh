#!/bin/bash
# Round 5: (1) the DDP / AMP / comm-hook / graph GPU tests on the default library,
# whose producer-side tail now waits for the previous bucket's collective only and
# joins the comm stream before its unpack; (2) the reduction / clip GPU tests on the
# one-level fused fold (GS_RED_ONE_LEVEL, its eight partial loads unconditional);
# (3) library variants against the default, two interleaved rounds: balanced
# reduction grid, one-level fold with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py tests/test_fused_norm_amp.py tests/test_amp_fused_ddp.py tests/test_gpu_comm_hooks.py tests/test_gpu_graphs.py tests/test_gpu_native_hook.py tests/test_gpu_clip_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_ddp.log 2>&1
rc=$?; tail -3 $OUT/pytest_ddp.log; [ $rc -ne 0 ] && exit $rc
GSYNC_LIB=$PWD/distributed_training_amd/lib/variants/onelevel/libgsync.so timeout -k 10 400 python -u -m pytest tests/test_clip_fold.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_onelevel.log 2>&1
rc=$?; tail -3 $OUT/pytest_onelevel.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS:-redbal onelevel onelevel_nb}" scripts/variant_rows.sh $OUT
