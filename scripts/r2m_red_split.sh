#!/bin/bash
# Per-kernel durations of the reductions (chunk kernel vs combine_partials)
# under rocprofv3 kernel-trace, R50 shapes, a few grid caps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2m; mkdir -p $OUT
for op in sqnorm unpacksq pack16; do
  for grid in default 2048 4096; do
    if [ $grid = default ]; then unset GS_RED_GRID; else export GS_RED_GRID=$grid; fi
    d=$OUT/${op}_$grid
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $d -o run -- python3 scripts/kernel_only.py resnet50 50 $op > $d.log 2>&1 || { echo "fail $op $grid"; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== $op grid=$grid"; cut -d, -f1-8 "$f" | head -6
    cp "$f" $OUT/${op}_${grid}_kernel_stats.csv
    t=$(find $d -name "*kernel_trace.csv" | head -1)
    python3 scripts/trace_gaps.py "$t" > $OUT/${op}_${grid}_gaps.txt && cat $OUT/${op}_${grid}_gaps.txt
    rm -rf $d
  done
done
