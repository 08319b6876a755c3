#!/bin/bash
# Diagnose the 4-rank gloo DDP rehearsal (tests/test_gpu_zz_bench.py::
# test_bench_multirank_gloo_rehearsal[ddp-4]) that went silent for 180 s: the same
# command with every rank's stacks dumped each 45 s (GSYNC_BENCH_TRACEBACK_S) into
# gpurun_out/, under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4n; mkdir -p $OUT
GSYNC_BENCH_TRACEBACK_S=45 timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 4 --pg-backend gloo --kernel-rates 0 \
  --model resnet18 --batch 16 --steps 3 --warmup 2 --cpu-baseline 0 > $OUT/ddp4.json 2> $OUT/ddp4.err
rc=$?; echo "rc=$rc"; tail -c 600 $OUT/ddp4.json; grep -E "^\[bench\]" $OUT/ddp4.err | tail -20
exit $rc
