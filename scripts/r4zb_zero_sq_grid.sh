#!/bin/bash
# The Σg² partials' grid inside configs[3]'s real ZeRO step (bf16 shard, 51 MB at
# one rank; scripts/zero_instep_sq.py): GS_RED_GRID default (2 Ki) / 1 Ki / 4 Ki /
# 8 Ki, interleaved, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4zb; mkdir -p $OUT
port=29671
for r in 1 2; do
  for g in default 1024 4096 8192; do
    port=$((port + 1))
    if [ $g = default ]; then unset GS_RED_GRID; else export GS_RED_GRID=$g; fi
    timeout -k 10 240 python -u scripts/zero_instep_sq.py $port >> $OUT/rows.jsonl 2>> $OUT/rows.err || { tail $OUT/rows.err; exit 1; }
  done
done
grep '^{' $OUT/rows.jsonl
