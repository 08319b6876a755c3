#!/bin/bash
# Kernel-trace durations of every grad-sync kernel alone on ResNet-50's
# parameters (rocprofv3 --kernel-trace --stats over 50 back-to-back launches):
# the kernel's own time, without the dispatch the launch timer's event pair adds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for op in pack pack16 unpack unpacksq sqnorm sqpart sgd adam; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/r3i_$op -o k -- python3 scripts/kernel_only.py resnet50 50 $op >> $OUT/r3i.log 2>&1 || { tail $OUT/r3i.log; exit 1; }
  s=$(find $OUT/r3i_$op -name "*kernel_stats.csv" | head -1); cp "$s" $OUT/r3i_${op}_kernel_stats.csv; rm -rf $OUT/r3i_$op
done
python3 - <<'PY'
import csv, json
B = {"pack": 8, "pack16": 6, "unpack": 8, "unpacksq": 8, "sqnorm": 4, "sqpart": 4, "sgd": 20, "adam": 28}
n = 25557032
out = {}
for op, b in B.items():
    rows = list(csv.DictReader(open(f"gpurun_out/r3i_{op}_kernel_stats.csv")))
    ks = {r["Name"][:60]: (int(r["Calls"]), float(r["AverageNs"])) for r in rows}
    main = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    tot_ns = sum(float(r["TotalDurationNs"]) for r in rows if "chunk_kernel" in r["Name"] or "combine" in r["Name"])
    calls = int(main["Calls"])
    us = tot_ns / calls / 1e3
    out[op] = {"kernel": main["Name"][:80], "calls": calls, "avg_us_all_launches": us,
               "frac": b * n / (us * 1e-6) / 8e12, "kernels": ks}
    print(op, round(us, 2), "us", round(out[op]["frac"], 3))
json.dump(out, open("gpurun_out/r3i_trace_rates.json", "w"), indent=1)
PY
