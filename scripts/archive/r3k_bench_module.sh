#!/bin/bash
# bench.py contract tests (N=1, N=2/3/4 gloo rehearsals with the post-timed legs,
# watchdog) and one N=1 bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_gpu_zz_bench.py -m gpu -x -v --timeout 700 --timeout-method thread > $OUT/r3k_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3k_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r3k_bench.json 2> $OUT/r3k_bench.err
rc=$?; tail -c 400 $OUT/r3k_bench.json; exit $rc
