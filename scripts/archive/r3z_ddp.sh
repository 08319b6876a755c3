#!/bin/bash
# the DDP GPU module (zero-size parameter, buffer hooks, CTA cap)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r3z_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3z_pytest.log; exit $rc
