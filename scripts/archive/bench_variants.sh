#!/bin/bash
# Bench variants, one after another, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
i=0
while IFS= read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  echo "== variant $i: $args" | tee -a $OUT/variants.log
  timeout -k 10 ${VT:-400} python -u bench.py --gpus 1 $args >> $OUT/variants.log 2>> $OUT/variants.err
  rc=$?
  echo "rc=$rc" | tee -a $OUT/variants.log
  tail -1 $OUT/variants.log
  if [ $rc -ne 0 ]; then tail -30 $OUT/variants.err; exit $rc; fi
done < "${1:-/dev/stdin}"
