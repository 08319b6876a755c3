"""From a rocprofv3 kernel_trace.csv: for each libgsync reduction launch
(chunk kernel followed by combine_partials), the chunk kernel's duration, the
gap to the combine, the combine's duration and the span start→end (µs,
medians over launches after the first 5)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
out = []
for a, b in zip(rows, rows[1:]):
    if "chunk_kernel" in a["Kernel_Name"] and "combine_partials" in b["Kernel_Name"]:
        s0, e0, s1, e1 = (int(a["Start_Timestamp"]), int(a["End_Timestamp"]),
                          int(b["Start_Timestamp"]), int(b["End_Timestamp"]))
        out.append((e0 - s0, s1 - e0, e1 - s1, e1 - s0))
solo = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "chunk_kernel" in r["Kernel_Name"]]
if out:
    out = out[5:] or out
    med = [statistics.median(x[k] for x in out) / 1e3 for k in range(4)]
    print("pairs %d  chunk %.2f us  gap %.2f us  combine %.2f us  span %.2f us" % (len(out), *med))
else:
    print("chunk kernels %d  median %.2f us" % (len(solo), statistics.median(solo[5:] or solo) / 1e3))
