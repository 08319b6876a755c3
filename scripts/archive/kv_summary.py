"""Summarise gpurun_out/kvariants.log: median GB/s per (model, kernel, variant)."""
import collections
import json
import statistics
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kvariants.log"):
    if line.startswith("=="):
        continue
    name, js = line.split(" ", 1)
    try:
        r = json.loads(js)
    except Exception:
        continue
    rows[(r["model"], r["replicas"], r["kernel"])][name].append(r["GBps"])
names = sorted({n for v in rows.values() for n in v})
print(f"{'':34s}" + "".join(f"{n[-10:]:>11s}" for n in names))
for k, v in rows.items():
    print(f"{k[0]:9s}x{k[1]} {k[2]:22s}" + "".join(f"{statistics.median(v[n]) if n in v else 0:11.0f}" for n in names))
