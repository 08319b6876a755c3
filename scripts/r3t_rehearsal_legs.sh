#!/bin/bash
# The driver's N>1 command, rehearsed at 4 ranks sharing the one GPU over gloo at full
# size, with every default leg (tail split, standalone collectives, parity, policy A/B,
# ZeRO-2 configs[3], Colossal configs[4]) under the leg watchdog
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
P=$((29500 + RANDOM % 1000))
GSYNC_BENCH_TRACEBACK_S=120 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port $P bench.py --gpus 4 --pg-backend gloo --steps 5 --warmup 2 \
  > $OUT/r3t_n4_gloo_legs.json 2> $OUT/r3t_n4_gloo_legs.err
rc=$?; echo "rc=$rc"; grep "\[bench\]" $OUT/r3t_n4_gloo_legs.err | tail -12
python3 -c "
import json; d=json.loads(open('$OUT/r3t_n4_gloo_legs.json').read().strip().splitlines()[-1])
print('value', d['value'], 'parity', d['parity']['ok'], 'legs', d.get('leg_seconds'), 'errors', d.get('leg_errors'), 'incomplete', d.get('legs_incomplete'))
for k in ('zero2', 'colossal'):
    if k in d: print(k, round(d[k]['images_per_sec'], 1), d[k]['parity']['ok'])
"
exit $rc
