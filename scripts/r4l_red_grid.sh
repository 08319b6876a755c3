#!/bin/bash
# Reduction grid caps (GS_RED_GRID) for unpack + Σg², Σg² and Σg² partials,
# interleaved, 2 rounds (scripts/red_grid_sweep.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4l; mkdir -p $OUT
for r in 1 2; do
  for cap in default 1024 2048 4096 8192; do
    if [ $cap = default ]; then unset GS_RED_GRID; else export GS_RED_GRID=$cap; fi
    timeout -k 10 200 python -u scripts/red_grid_sweep.py >> $OUT/red_grid.jsonl 2>> $OUT/red_grid.err || { tail $OUT/red_grid.err; exit 1; }
  done
done
unset GS_RED_GRID
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4l/red_grid.jsonl"):
    r = json.loads(l)
    agg[(r["model"], r["kernel"], r["GS_RED_GRID"])].append(round(r["frac"], 4))
for k in sorted(agg):
    print(k, agg[k])
PY
