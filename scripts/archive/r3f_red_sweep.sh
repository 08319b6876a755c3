#!/bin/bash
# Σg² (sqnorm / sqnorm_partial) grid and group-size sweep, interleaved, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for v in libgsync variants/libgsync_red4 variants/libgsync_red8; do
    for grid in 0 1024 4096 8192; do
      if [ $grid = 0 ]; then unset GS_RED_GRID; else export GS_RED_GRID=$grid; fi
      GSYNC_LIB=distributed_training_amd/lib/$v.so timeout -k 10 200 python -u scripts/kernel_rates.py resnet50 "$(basename $v)_grid$grid" >> $OUT/r3f_red.jsonl 2>> $OUT/r3f_red.err || { tail $OUT/r3f_red.err; exit 1; }
    done
  done
done
unset GS_RED_GRID
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r3f_red.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[r["label"]].append(r)
for k, rs in agg.items():
    keys = ["sqnorm_f32", "sqnorm_partial_f32", "clip_path_sgd", "unpack_f32+sqnorm", "pack_f32_to_bf16"]
    print(k, {x: round(sum(r["frac"][x] for r in rs) / len(rs), 4) for x in keys})
PY
