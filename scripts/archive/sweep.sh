#!/bin/bash
# task-size x build-variant sweep (scripts/sweep_tasks.py), rows -> gpurun_out/sweep.jsonl
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for lib in distributed_training_amd/lib/libgsync.so distributed_training_amd/lib/variants/*.so; do
  for MR in ${MODELS:-resnet50:1 resnet18:1 resnet152:2}; do
    GSYNC_LIB=$lib timeout -k 10 150 python -u scripts/sweep_tasks.py --model ${MR%%:*} --replicas ${MR#*:} \
      --tag $(basename $lib .so) ${SWEEP_ARGS:-} >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || exit 1
  done
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/sweep.jsonl") if l.startswith("{")]
t=collections.defaultdict(dict)
for r in rows: t[(r["tag"],r["model"],r["replicas"],r["op"])][r["req"]]=round(r["GBps"])
for k,v in sorted(t.items()): print(*k, v)
PY
