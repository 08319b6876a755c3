set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ddp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_k.log 2>&1; tail -1 gpurun_out/pt_k.log
for il in 1 0 1 0; do
  GS_INTERLEAVE=$il timeout -k 10 200 python -u scripts/copy_ceiling.py | sed "s/^{/{\"tag\": \"il$il\", /" >> gpurun_out/pack_ceiling.jsonl || exit 1
  for MR in resnet50:1 resnet152:2; do
    GS_INTERLEAVE=$il timeout -k 10 150 python -u scripts/sweep_tasks.py --model ${MR%%:*} --replicas ${MR#*:} --tasks 0 --rounds 10 --ops pack,unpack,sgd,adam --tag il$il >> gpurun_out/pack_sweep.jsonl 2>> gpurun_out/pack_sweep.err || exit 1
  done
done
