#!/bin/bash
# ZeRO engine on the C++ hooks: GPU parity tests, then the reference's DeepSpeed
# workload (ResNet-18 / CIFAR, bf16, ZeRO-2, batch 96) with the C++ and the Python hooks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_zero.py tests/test_gpu_native_hook.py tests/test_gpu_amp_nosync.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/r3l_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3l_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/zero_host.py --steps 100 --out $OUT/r3l_zero_host.jsonl > $OUT/r3l.log 2>&1 || { tail $OUT/r3l.log; exit 1; }
GSYNC_NATIVE_HOOK=0 timeout -k 10 400 python -u scripts/zero_host.py --steps 100 --impls zero2 --out $OUT/r3l_zero_host.jsonl >> $OUT/r3l.log 2>&1 || { tail $OUT/r3l.log; exit 1; }
cat $OUT/r3l_zero_host.jsonl
