"""From a rocprofv3 kernel_trace.csv of `bench.py`: per libgsync kernel, the
durations of its launches in the timed region (the last `steps` launches of
the update kernel, the same count per step for the others), to set beside
bench.py's HIP-event figure for the same launches.
    python scripts/trace_roofline.py <kernel_trace.csv> <steps> <out.json>"""
import csv
import json
import re
import statistics
import sys

path, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    m = re.search(r"chunk_kernel<gs::\(anonymous namespace\)::(\w+)<", r["Kernel_Name"])
    if "chunk_kernel" in r["Kernel_Name"] and m:
        by.setdefault(m.group(1), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
res = {}
upd = by.get("SgdOp") or by.get("AdamOp") or []
for k, v in by.items():
    per_step = max(1, round(len(v) / max(1, len(upd)))) if upd else 1
    last = v[-steps * per_step:]
    res[k] = {"launches_total": len(v), "timed_region_launches": len(last),
              "avg_us": statistics.fmean(last), "median_us": statistics.median(last)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
