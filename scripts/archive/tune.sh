#!/bin/bash
# Kernel tuning sweep: task sizing (env) x build variants, bench_kernels.py
# rows appended to gpurun_out/tune.jsonl.  Each run has its own time limit.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
run() {  # tag env... -- model replicas
  local tag=$1; shift
  echo "== $tag $*" >> $OUT/tune.log
  env "$@" timeout -k 10 150 python -u bench_kernels.py --skip-torch --iters 30 --tag "$tag" --model $M --replicas $R \
     >> $OUT/tune.jsonl 2>> $OUT/tune.err
}
for MR in ${MODELS:-resnet50:1 resnet152:2}; do
  M=${MR%%:*}; R=${MR#*:}
  run auto GSYNC_LIB=distributed_training_amd/lib/libgsync.so || exit 1
  run fixed4096 GS_TASK_UNITS=4096 || exit 1
  run fixed1024 GS_TASK_UNITS=1024 || exit 1
  run target1024 GS_TARGET_TASKS=1024 || exit 1
  run target2040 GS_TARGET_TASKS=2040 || exit 1
  run target3840 GS_TARGET_TASKS=3840 || exit 1
  for v in distributed_training_amd/lib/variants/*.so; do
    run $(basename $v .so) GSYNC_LIB=$v || exit 1
  done
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/tune.jsonl") if l.startswith("{")]
t=collections.defaultdict(dict)
for r in rows: t[(r["model"],r["replicas"],r["tag"])][r["kernel"]]=round(r["GBps"])
for k,v in t.items(): print(*k, v)
PY
