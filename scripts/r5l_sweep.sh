#!/bin/bash
# Round 5: the Σg² at ResNet-50 against a plain read stream of the same bytes
# (scripts/micro/read_ceiling.hip: 14.1-15.1 µs cached, 13.5 µs NT on a 2 Ki
# grid-stride grid, against the library's ~18 µs).  Variants against the
# default, two interleaved rounds: pf1 (the next group's chunk entries fetched
# one iteration ahead, GS_CHUNK_PREFETCH), ntsq (non-temporal Σg² loads below
# the cache size, GS_NT_SQNORM=1), both.  First the reduction GPU tests on pf1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5l; mkdir -p $OUT
export TMPDIR=/tmp
GSYNC_LIB=$PWD/distributed_training_amd/lib/variants/pf1/libgsync.so timeout -k 10 400 python -u -m pytest tests/test_clip_fold.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_pf1.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_pf1.log; [ $rc -ne 0 ] && exit $rc
export ENV_ntsq="GS_NT_SQNORM=1"
VARIANTS="${VARIANTS:-pf1 ntsq}" scripts/variant_rows.sh $OUT
