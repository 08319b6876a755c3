#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_zero.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/r3r_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3r_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/zero_graph.py --steps 100 --deterministic 0 > $OUT/r3r_zero_graph.jsonl 2> $OUT/r3r.err || { tail $OUT/r3r.err; exit 1; }
cat $OUT/r3r_zero_graph.jsonl
