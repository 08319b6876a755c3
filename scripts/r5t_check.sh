#!/bin/bash
# Round 5: the producer-side tail's collective watched through its unpack's own
# stop event (no watchdog event packet after it): the communicator / DDP GPU
# tests, two default bench runs (legs off) for the tail split, and the kernel
# trace of the end of backward (scripts/tail_trace.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5t}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_comm_api.py tests/test_gpu_one_comm.py tests/test_gpu_ddp.py tests/test_gpu_native_hook.py tests/test_gpu_comm_hooks.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="" scripts/variant_rows.sh $OUT || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/prof -o tail -- python3 -u scripts/tail_trace.py run > $OUT/run.log 2>&1 || { tail -30 $OUT/run.log; exit 1; }
python3 scripts/tail_trace.py analyze $(find $OUT/prof -name "*kernel_trace.csv" | head -1) > $OUT/tail.jsonl
rm -rf $OUT/prof
echo done
