#!/bin/bash
# the 4-rank full-size rehearsal (ResNet-50 x256, 4 ranks sharing
# the one GPU over gloo), once, with every rank's stacks dumped periodically; then
# the no-libgsync reproduction of the stall it hit (scripts/gloo_cuda_repro.py):
# MODE=cpu (host staging, the fix) and last MODE=hook (gloo's own CUDA path from
# the autograd thread, expected to deadlock: its own time limit ends the call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export OUT
P=$((29500 + RANDOM % 1000))
GSYNC_BENCH_TRACEBACK_S=60 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port $P bench.py --gpus 4 --pg-backend gloo --steps 5 --warmup 2 \
  --cpu-baseline 0 --kernel-rates 0 > $OUT/r3e_n4_gloo_r50.json 2> $OUT/r3e_n4_gloo_r50.err
rc=$?; echo "rehearsal rc=$rc"; tail -3 $OUT/r3e_n4_gloo_r50.err; [ $rc -ne 0 ] && exit $rc
python3 -c "import json; d=json.loads(open('$OUT/r3e_n4_gloo_r50.json').read().strip().splitlines()[-1]); print('value', d['value'], 'parity', d['parity']['ok'], 'ab', d.get('bucket_policy_ab', {}).get('decision'))"
P=$((30600 + RANDOM % 1000))
MODE=cpu TB_S=45 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port $P scripts/gloo_cuda_repro.py > $OUT/r3e_repro_cpu.log 2>&1
rc=$?; echo "repro cpu rc=$rc"; tail -3 $OUT/r3e_repro_cpu.log; [ $rc -ne 0 ] && exit $rc
P=$((31700 + RANDOM % 1000))
MODE=hook TB_S=45 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port $P scripts/gloo_cuda_repro.py > $OUT/r3e_repro_hook.log 2>&1
echo "repro hook rc=$? (124 = deadlocked until the time limit)"; tail -5 $OUT/r3e_repro_hook.log
exit 0
