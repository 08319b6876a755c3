#!/bin/bash
# Full -m gpu suite then smoke, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r2}
# bench children of tests/test_gpu_zz_bench.py stream their stderr here (progress the box can see)
export GSYNC_TEST_PROGRESS_DIR=$OUT/${TAG}_progress
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/${TAG}_pytest_gpu.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $OUT/${TAG}_pytest_gpu.log | tail -60; tail -3 $OUT/${TAG}_pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()"
