#!/bin/bash
# In-step A/B of the update-plan task size (GSYNC_UPDATE_TASK_UNITS 512 vs 0 =
# library default), interleaved on one box.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for tu in ${TUS:-512 0}; do
    echo "== tu=$tu round $r" >> $OUT/ab_update.log
    GSYNC_UPDATE_TASK_UNITS=$tu timeout -k 10 400 python -u bench.py --cpu-baseline 0 ${BENCH_ARGS:-} >> $OUT/ab_update.log 2>> $OUT/ab_update.err || exit 1
  done
done
