#!/bin/bash
# Fused SGD / Adam beyond the Infinity Cache (ResNet-152 x 2) and on ResNet-50:
# update-kernel variants (group size G, non-temporal loads of the grad stream or of
# every stream), interleaved, 2 rounds; plan launch timer, 30 launches each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4b; mkdir -p $OUT
for r in 1 2; do
  for v in libgsync ${VARIANTS:-variants/libgsync_sgd4 variants/libgsync_ntg variants/libgsync_sgd4ntg variants/libgsync_ntall variants/libgsync_sgd8}; do
    for m in resnet152:2 resnet50:1; do
      GSYNC_LIB=distributed_training_amd/lib/$v.so timeout -k 10 200 python -u bench_kernels.py --model ${m%%:*} --replicas ${m#*:} --skip-torch --iters 30 --tag "$(basename $v)" >> $OUT/update.jsonl 2>> $OUT/update.err || { tail $OUT/update.err; exit 1; }
    done
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4b/update.jsonl"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    if r.get("impl") == "libgsync":
        agg[(r["kernel"], r["model"], r["replicas"], r["tag"])].append(r["frac_of_8TBps"])
for k in sorted(agg, key=str):
    v = agg[k]
    print(k, [round(x, 4) for x in v], "mean", round(sum(v) / len(v), 4))
PY
