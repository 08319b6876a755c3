#!/bin/bash
# Overlapped optimizer: GPU tests, then bench with / without it (one box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2r; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_c_abi.py -m gpu -x -v --timeout 120 --timeout-method thread -k "overlapped or plain_c or ws1_rccl_grads" > $OUT/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
for v in "" "--optimizer-overlap 1" "--optimizer-overlap 1 --grad-as-bucket-view"; do
  tag=$(echo "x$v" | tr -c 'a-z0-9' '_')
  timeout -k 10 400 python -u bench.py --cpu-baseline 0 --kernel-rates 0 $v > $OUT/b$tag.json 2> $OUT/b$tag.err || { tail -5 $OUT/b$tag.err; exit 1; }
  grep '^{' $OUT/b$tag.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grad_sync']; t=g.get('tail_ms') or {}
print(json.dumps({'args': '''$v''', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'upd_ms_per_step': d['roofline']['avg_launch_ms'],
 'upd_frac': d['roofline']['frac'], 'tail_timed_ms': t.get('total_timed_step'),
 'tail_split': {k: t.get(k) for k in ('total','queue','pack','collective','unpack')}, 'parity_ok': (d.get('parity') or {}).get('ok')}))" | tee -a $OUT/summary.jsonl
done
