#!/bin/bash
# configs[3] (bf16 ResNet-50 on the ZeRO-2 engine): channels_last vs NCHW —
# the bf16 model's BatchNorm runs torch's native kernels (MIOpen BN needs fp32
# weights), whose channels_last path dominated the r3u profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
A="--engine zero2 --steps 10 --warmup 3 --kernel-rates 0 --parity 0 --cpu-baseline 0"
timeout -k 10 400 python -u bench.py $A > $OUT/r3x_zero_cl.json 2> $OUT/r3x_zero_cl.err || exit $?
timeout -k 10 400 python -u bench.py $A --no-channels-last > $OUT/r3x_zero_nchw.json 2> $OUT/r3x_zero_nchw.err || exit $?
for f in cl nchw; do python -c "import json,sys; d=json.loads(open('$OUT/r3x_zero_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
