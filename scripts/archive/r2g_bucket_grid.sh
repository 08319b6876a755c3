#!/bin/bash
# In-step bucket kernels share the CUs with MIOpen's backward: does a smaller
# pack / unpack grid (GSYNC_BUCKET_GRID) trade bucket-kernel time for backward
# time?  bench.py at N=1, interleaved rounds, 40 timed steps each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2bg; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline 0 --kernel-rates 0 --parity 0 > /dev/null 2> $OUT/compile.err || exit 1
for round in 1 2 3; do
  for gr in 0 256 512 1024 2048; do
    GSYNC_BUCKET_GRID=$gr timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --cpu-baseline 0 --kernel-rates 0 --parity 0 > $OUT/g${gr}_$round.json 2> $OUT/g${gr}_$round.err || { tail -3 $OUT/g${gr}_$round.err; exit 1; }
    grep '^{' $OUT/g${gr}_$round.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grad_sync']
print(json.dumps({'bucket_grid': $gr, 'round': $round, 'value': round(d['value'],1), 'ms_per_step': round(d['ms_per_step'],3), 'tail_us': round(g['tail_ms']['total_timed_step']*1e3,1), 'pack_last_us': round(g['tail_ms']['pack']*1e3,1)}))" | tee -a $OUT/summary.jsonl
  done
done
