#!/bin/bash
# Round-2 extras: full -m gpu suite + smoke, a roctx marker trace of the bench
# (GSYNC_ROCTX=1, marker + kernel trace, summaries only), then the
# MIOpen-Find (cudnn.benchmark) experiment under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r2h}
export TMPDIR=/tmp
TAG=$TAG bash scripts/gpu_tests.sh || exit $?
echo "== roctx marker trace"
GSYNC_ROCTX=1 timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats -f csv -d $OUT/mk_$TAG -o bench -- python3 -u bench.py --steps 3 --warmup 2 --cpu-baseline 0 --parity 0 > $OUT/${TAG}_marker_bench.json 2> $OUT/${TAG}_marker.err || { tail -20 $OUT/${TAG}_marker.err; exit 1; }
for f in $(find $OUT/mk_$TAG -name "*stats*.csv"); do cp $f $OUT/${TAG}_marker_$(basename $f); done
python3 - $OUT/mk_$TAG $OUT/${TAG}_marker_ranges.json <<'PY'
import csv, glob, json, os, sys, collections
rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*marker_api_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    name = r.get("Function") or r.get("Name") or r.get("Operation") or "?"
    try:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    except Exception:
        continue
    agg[name][0] += 1
    agg[name][1] += d
json.dump({k: {"count": v[0], "host_us_total": v[1]} for k, v in sorted(agg.items())}, open(sys.argv[2], "w"), indent=1)
print(json.dumps({k: v[0] for k, v in agg.items()}))
PY
rm -rf $OUT/mk_$TAG
echo "== MIOpen Find experiment (cudnn.benchmark=1)"
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 --cudnn-benchmark 1 --cpu-baseline 0 --parity 0 > $OUT/${TAG}_bench_find.json 2> $OUT/${TAG}_bench_find.err
echo "find rc=$?"; cat $OUT/${TAG}_bench_find.json | cut -c1-300; grep "warmup step" $OUT/${TAG}_bench_find.err
