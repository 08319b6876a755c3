#!/bin/bash
# Group size of the 16-bit packs (GS_G_PACK16_16 for bf16 -> bf16, GS_G_PACK16 for
# fp32 -> bf16): library variants, interleaved, 2 rounds (scripts/pack16_sweep.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4k; mkdir -p $OUT
for r in 1 2; do
  for v in libgsync ${VARIANTS:-variants/libgsync_p16g1 variants/libgsync_p16g2 variants/libgsync_p16g4 variants/libgsync_p16g16}; do
    GSYNC_LIB=distributed_training_amd/lib/$v.so timeout -k 10 200 python -u scripts/pack16_sweep.py >> $OUT/pack16.jsonl 2>> $OUT/pack16.err || { tail $OUT/pack16.err; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4k/pack16.jsonl"):
    r = json.loads(l)
    agg[(r["model"], r["src"], r["lib"])].append(round(r["frac"], 4))
for k in sorted(agg):
    print(k, agg[k])
PY
