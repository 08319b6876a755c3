#!/bin/bash
# bench.py variants on one box (each under its own limit; a failure ends the run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2p; mkdir -p $OUT
i=0
while IFS= read -r v; do
  i=$((i+1))
  echo "== $i: $v"
  timeout -k 10 400 python -u bench.py --cpu-baseline 0 --kernel-rates 0 $v > $OUT/v$i.json 2> $OUT/v$i.err || { tail -5 $OUT/v$i.err; exit 1; }
  grep '^{' $OUT/v$i.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grad_sync']; t=g.get('tail_ms') or {}
print(json.dumps({'args': '''$v''', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'opt_ms': d['roofline']['avg_launch_ms'],
 'tail_timed_ms': t.get('total_timed_step'), 'tail_split': {k: t.get(k) for k in ('total','queue','pack','collective','unpack')},
 'parity_ok': (d.get('parity') or {}).get('ok')}))" | tee -a $OUT/summary.jsonl
done <<'LIST'

--grad-as-bucket-view
--last-bucket-cap-mb 1
--graph 1
--bucket-dtype bf16
LIST
