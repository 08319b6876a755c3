#!/bin/bash
# The Σg² load policy inside configs[3]'s real step (scripts/zero_instep_sq.py):
# GS_NT_SQNORM 0 / 1 / 2, interleaved, 3 rounds, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4v; mkdir -p $OUT
port=29641
for r in 1 2 3; do
  for pol in 0 1 2; do
    port=$((port + 1))
    GS_NT_SQNORM=$pol timeout -k 10 240 python -u scripts/zero_instep_sq.py $port >> $OUT/rows.jsonl 2>> $OUT/rows.err || { tail $OUT/rows.err; exit 1; }
  done
done
grep '^{' $OUT/rows.jsonl
