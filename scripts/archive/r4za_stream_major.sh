#!/bin/bash
# Stream-major load issue in the updates (GS_STREAM_MAJOR) and the SGD's group of 4
# (GS_G_SGD) as library variants (built with make EXTRA_DEFS=... into
# distributed_training_amd/lib/variants/<name>/), interleaved, 2 rounds
# (scripts/update_rows.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4za; mkdir -p $OUT
for r in 1 2; do
  for v in default sm smg4 g4; do
    lib=distributed_training_amd/lib/libgsync.so
    [ $v != default ] && lib=distributed_training_amd/lib/variants/$v/libgsync.so
    GSYNC_LIB=$lib ROWS_LABEL=$v timeout -k 10 200 python -u scripts/update_rows.py >> $OUT/rows.jsonl 2>> $OUT/rows.err || { tail $OUT/rows.err; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4za/rows.jsonl"):
    r = json.loads(l)
    agg[(r["set"], r["kernel"], r["variant"])].append(round(r["frac"], 4))
for k in sorted(agg):
    print(k, agg[k])
PY
