"""From a rocprofv3 kernel_trace.csv of the driver's `bench.py` command: the
durations of the launches behind the line's `roofline`, to set beside the plan
launch timer's figures for the same launches (bench.py `_trace_check`).

* ``SgdOp``: the fused SGD of the timed steps (launches W .. W+K-1 of the run:
  W warm-up steps, then K timed ones, one update launch each);
* ``SgdOp_beyond_ic``: the same kernel on the ResNet-152 x 2 working set
  (grad_sync_kernels.beyond_ic's `sgd_momentum_wd` row: 3 warm + `iters` timed
  launches, the first of the run's SGD launches longer than 3x the in-step median);
* every other libgsync chunk kernel: count and average over the whole run.

    python scripts/trace_bench.py <kernel_trace.csv> <warmup> <steps> <iters> <run label> <out.json>
"""
import csv
import json
import re
import statistics
import sys

path, warm, steps, iters, label, out = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]),
                                        sys.argv[5], sys.argv[6])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    m = re.search(r"chunk_kernel<gs::\(anonymous namespace\)::(\w+)<", r["Kernel_Name"])
    if m:
        by.setdefault(m.group(1), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def summary(v, what):
    return {"avg_us": statistics.fmean(v), "median_us": statistics.median(v), "timed_region_launches": len(v),
            "what": what, "run": label}


res = {}
sgd = by.get("SgdOp", [])
if len(sgd) >= warm + steps:
    ins = sgd[warm:warm + steps]
    res["SgdOp"] = summary(ins, f"launches {warm}..{warm + steps - 1}: the timed steps' fused SGD (ResNet-50)")
    med = statistics.median(ins)
    big = [d for d in sgd[warm + steps:] if d > 3 * med]
    if len(big) >= 3 + iters:
        res["SgdOp_beyond_ic"] = summary(big[3:3 + iters], "grad_sync_kernels.beyond_ic sgd_momentum_wd row "
                                                           "(ResNet-152 x 2), its timed launches")
for k, v in by.items():
    res.setdefault("all", {})[k] = {"launches": len(v), "avg_us": statistics.fmean(v)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "all"}))
