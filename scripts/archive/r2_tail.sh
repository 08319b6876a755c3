#!/bin/bash
# The exposed end-of-backward tail, A/B: the last bucket's chain on the
# producer stream (default) vs on the comm stream (GSYNC_TAIL_ON_PRODUCER=0),
# with and without a 1 MiB last bucket; GPU tests of the paths it touches first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r2k}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_zero.py tests/test_gpu_graphs.py tests/test_gpu_amp_nosync.py -x -q --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
for tp in 1 0; do
for cap in none 1; do
  echo "== bench tail_on_producer=$tp last-bucket cap $cap"
  extra=""; [ $cap != none ] && extra="--last-bucket-cap-mb $cap"
  GSYNC_TAIL_ON_PRODUCER=$tp timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-rates 0 $extra > $OUT/${TAG}_bench_tp${tp}_cap_$cap.json 2> $OUT/${TAG}_bench_tp${tp}_cap_$cap.err || { tail -20 $OUT/${TAG}_bench_tp${tp}_cap_$cap.err; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/${TAG}_bench_tp${tp}_cap_$cap.json') if l.startswith('{')][0]
print(round(d['value'],1), round(d['ms_per_step'],3), d['grad_sync']['tail_ms'], d['parity']['ok'])"
done
done
