#!/bin/bash
# rocprofv3 kernel trace of the update rows (scripts/update_rows.py: SGD and Adam
# at ResNet-50 and ResNet-152 x 2, 23 launches each) beside the plan launch
# timer's own numbers from the same run: the trace's per-launch durations of the
# beyond-cache launches against the timer behind roofline.frac_beyond_ic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4zc; mkdir -p $OUT
ROWS_LABEL=trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o upd -- python3 -u scripts/update_rows.py > $OUT/rows.jsonl 2> $OUT/rows.err || { tail $OUT/rows.err; exit 1; }
python3 - <<'PY'
import csv, glob, json
tr = glob.glob("gpurun_out/r4zc/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(tr))]
out = {}
for kind in ("SgdOp", "AdamOp"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if kind in r["Kernel_Name"]]
    # launch order: ResNet-50 23 launches (3 warm + 20 timed), then ResNet-152 x 2 23 launches
    out[kind] = {"resnet50_timed_avg_us": sum(d[3:23]) / 20, "resnet152x2_timed_avg_us": sum(d[26:46]) / 20, "launches": len(d)}
timer = [json.loads(l) for l in open("gpurun_out/r4zc/rows.jsonl") if l.startswith("{")]
for t in timer:
    k = "SgdOp" if t["kernel"].startswith("sgd") else "AdamOp"
    out[k]["timer_%s_avg_us" % t["set"]] = t["avg_ms"] * 1e3
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/r4zc/trace_vs_timer.json", "w"), indent=1)
PY
for f in $(find $OUT/prof -name "*stats*.csv"); do cp $f $OUT/$(basename $f); done
rm -rf $OUT/prof
