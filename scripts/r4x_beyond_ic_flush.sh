#!/bin/bash
# Beyond-cache update rows back to back vs with a 1 GiB read between launches
# (scripts/beyond_ic_flush.py), 2 rounds in one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4x; mkdir -p $OUT
timeout -k 10 200 python -u scripts/beyond_ic_flush.py > $OUT/flush.jsonl 2> $OUT/flush.err || { tail $OUT/flush.err; exit 1; }
cat $OUT/flush.jsonl
