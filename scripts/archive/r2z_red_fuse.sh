#!/bin/bash
# A/B of the reduction combine: combine_partials launch (GS_RED_FUSE=0) vs the
# in-kernel two-level ticket over R groups (GS_RED_FUSE=R).  Correctness first
# (scripts/red_fuse_check.py for every R, the kernel GPU tests at the largest),
# then rocprofv3 kernel-trace durations over R and the reduction grid cap, and
# the plan-timer rates (bench_kernels.py, R50 and R152x2).  Every GPU step has
# its own limit; the first failure ends the script.
#   env: RS="0 8 16 32 64" GRIDS="default 2048 4096" KB=1 TAG=r2z
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r2z}
OUT=gpurun_out/$TAG; mkdir -p $OUT
RS=${RS:-"0 8 16 32 64"}
GRIDS=${GRIDS:-"default 2048 4096"}
for f in $RS; do
  GS_RED_FUSE=$f timeout -k 10 120 python3 -u scripts/red_fuse_check.py > $OUT/check_fuse$f.jsonl 2>&1 || { tail -20 $OUT/check_fuse$f.jsonl; exit 1; }
done
last=${RS##* }
GS_RED_FUSE=$last timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_amp_nosync.py tests/test_amp_fused_ddp.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_fuse$last.log 2>&1 || { tail -30 $OUT/pytest_fuse$last.log; exit 1; }
tail -1 $OUT/pytest_fuse$last.log
for f in $RS; do
  for grid in $GRIDS; do
    if [ $grid = default ]; then unset GS_RED_GRID; else export GS_RED_GRID=$grid; fi
    d=$OUT/sq_f${f}_$grid
    GS_RED_FUSE=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $d -o run -- python3 scripts/kernel_only.py resnet50 50 sqnorm > $d.log 2>&1 || { echo "fail $f $grid"; tail $d.log; exit 1; }
    t=$(find $d -name "*kernel_trace.csv" | head -1)
    python3 scripts/trace_gaps.py "$t" > $OUT/sq_f${f}_${grid}_gaps.txt && echo "R=$f grid=$grid: $(cat $OUT/sq_f${f}_${grid}_gaps.txt)"
    rm -rf $d
  done
done
unset GS_RED_GRID
if [ "${KB:-1}" == "1" ]; then
  for f in $RS; do
    GS_RED_FUSE=$f timeout -k 10 300 python3 -u bench_kernels.py --model resnet50 --replicas 1 --iters 50 --skip-torch > $OUT/kb_r50_fuse${f}.jsonl 2> $OUT/kb.err || { tail $OUT/kb.err; exit 1; }
    GS_RED_FUSE=$f timeout -k 10 300 python3 -u bench_kernels.py --model resnet152 --replicas 2 --iters 50 --skip-torch > $OUT/kb_r152x2_fuse${f}.jsonl 2>> $OUT/kb.err || { tail $OUT/kb.err; exit 1; }
  done
  python3 - "$OUT" <<'EOF'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/kb_*.jsonl")):
    for l in open(f):
        if not l.startswith("{"):
            continue
        d = json.loads(l)
        if d.get("impl") == "libgsync" and "sq" in d["kernel"]:
            print(f.split("/")[-1], d["kernel"], "%.2f us" % (d["avg_ms"] * 1e3), "%.0f GB/s" % d["GBps"])
EOF
fi
echo "== done"
