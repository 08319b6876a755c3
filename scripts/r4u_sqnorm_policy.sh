#!/bin/bash
# GS_NT_SQNORM 0 (cached) / 1 (NT, the default) / 2 (NT above the cache size) on
# bench.py's own kernel rows, the ZeRO N=8-shard clip path and the clip chain
# (scripts/sqnorm_policy_rows.py), interleaved, 3 rounds, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4u; mkdir -p $OUT
port=29611
for r in 1 2 3; do
  for pol in 0 1 2; do
    port=$((port + 1))
    GS_NT_SQNORM=$pol timeout -k 10 200 python -u scripts/sqnorm_policy_rows.py $port >> $OUT/rows.jsonl 2>> $OUT/rows.err || { tail $OUT/rows.err; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4u/rows.jsonl"):
    r = json.loads(l)
    agg[(r["row"], r["GS_NT_SQNORM"])].append(round(r.get("frac", 0) or r["avg_ms"] * 1e3, 4))
for k in sorted(agg):
    print(k, agg[k])
PY
