#!/bin/bash
# Update-kernel group size / grid sweep (Adam G 2/4/8, SGD G 2/4; GS_MAX_GRID),
# ResNet-50 and ResNet-152 x2 (beyond the 256 MB Infinity Cache), interleaved, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for v in libgsync variants/libgsync_adam2 variants/libgsync_adam8 variants/libgsync_sgd4; do
    for grid in 0 2048 4096; do
      if [ $grid = 0 ]; then unset GS_MAX_GRID; else export GS_MAX_GRID=$grid; fi
      for m in resnet50:1 resnet152:2; do
        GSYNC_LIB=distributed_training_amd/lib/$v.so timeout -k 10 200 python -u bench_kernels.py --model ${m%%:*} --replicas ${m#*:} --skip-torch --iters 30 --tag "$(basename $v)_grid$grid" >> $OUT/r3j_update.jsonl 2>> $OUT/r3j.err || { tail $OUT/r3j.err; exit 1; }
      done
    done
  done
done
unset GS_MAX_GRID
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r3j_update.jsonl"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    if r.get("kernel") in ("sgd_momentum_wd", "adam") and r.get("impl") == "libgsync":
        agg[(r["tag"], r["model"], r["replicas"], r["kernel"])].append((r["frac_of_8TBps"], r.get("batched_frac_of_8TBps", 0)))
for k in sorted(agg, key=str):
    v = agg[k]
    print(k, "per-launch", round(sum(a for a, _ in v) / len(v), 4), "batched", round(sum(b for _, b in v) / len(v), 4))
PY
