#!/bin/bash
# The plain-stream probe with stream-major load issue (scripts/micro/stream_mix.hip
# *_streammajor cases) beside access-major, one box, one process (2 rounds inside).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4z; mkdir -p $OUT
timeout -k 10 180 scripts/micro/stream_mix > $OUT/stream_mix.jsonl || exit 1
grep -E '"sgd3r2w_g(2|4)_ntl|adam4r3w_g4_ntl' $OUT/stream_mix.jsonl
