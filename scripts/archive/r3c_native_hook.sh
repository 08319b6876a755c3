set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_hook.py tests/test_gpu_ddp.py tests/test_gpu_graphs.py tests/test_gpu_one_comm.py tests/test_clip_fold.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3c_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r3c_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/cifar_host.py --steps 100 --out gpurun_out/r3c_cifar_host.jsonl > gpurun_out/r3c_cifar.log 2>&1 || { tail -20 gpurun_out/r3c_cifar.log; exit 1; }
GSYNC_NATIVE_HOOK=0 timeout -k 10 300 python -u scripts/cifar_host.py --steps 100 --impls gsync --out gpurun_out/r3c_cifar_host_pyhook.jsonl >> gpurun_out/r3c_cifar.log 2>&1 || { tail -20 gpurun_out/r3c_cifar.log; exit 1; }
cat gpurun_out/r3c_cifar_host.jsonl gpurun_out/r3c_cifar_host_pyhook.jsonl
