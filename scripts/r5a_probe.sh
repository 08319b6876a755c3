#!/bin/bash
# Round 5 first box call: the stream-packet probe (scripts/micro/event_chain.hip)
# and the driver's bench with configs[3] / configs[4] legs forced on at N=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 90 scripts/micro/event_chain > $OUT/event_chain.jsonl 2> $OUT/event_chain.err || { cat $OUT/event_chain.err; exit 1; }
cat $OUT/event_chain.jsonl
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 --zero-leg 1 --colossal-leg 1 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print(d['value'], d.get('leg_seconds'), d.get('leg_errors'), d.get('warmup_s'))
for k in ('zero2','colossal'):
    print(k, json.dumps(d.get(k))[:1500])
"
