#!/bin/bash
# Host-side enqueue ranges of the bucket path (roctx marker trace, summaries
# only) and the exposed tail with / without a capped last bucket (N=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r2i}
export TMPDIR=/tmp
echo "== roctx marker trace"
GSYNC_ROCTX=1 timeout -k 10 600 rocprofv3 --marker-trace --stats -f csv -d $OUT/mk_$TAG -o bench -- python3 -u bench.py --steps 3 --warmup 2 --cpu-baseline 0 --parity 0 > $OUT/${TAG}_marker_bench.json 2> $OUT/${TAG}_marker.err || { tail -20 $OUT/${TAG}_marker.err; exit 1; }
python3 - $OUT/mk_$TAG $OUT/${TAG}_marker_ranges.json <<'PY'
import csv, glob, json, os, sys, collections
rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*marker_api_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    name = r.get("Function") or r.get("Name") or "?"
    try:
        agg[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    except Exception:
        pass
out = {k: {"count": len(v), "host_us_total": sum(v), "host_us_max": max(v), "host_us_median": sorted(v)[len(v) // 2]}
       for k, v in sorted(agg.items())}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
PY
rm -rf $OUT/mk_$TAG
for cap in none 1; do
  echo "== bench last-bucket cap $cap"
  extra=""; [ $cap != none ] && extra="--last-bucket-cap-mb $cap"
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 $extra > $OUT/${TAG}_bench_cap_$cap.json 2> $OUT/${TAG}_bench_cap_$cap.err || { tail -20 $OUT/${TAG}_bench_cap_$cap.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/${TAG}_bench_cap_$cap.json')); print(d['value'], d['ms_per_step'], d['grad_sync']['tail_ms'], d['grad_sync']['bucket_bytes'], d['parity']['ok'])"
done
