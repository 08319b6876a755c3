"""GPU busy fraction of the last `steps` seconds-window in a rocprofv3 kernel trace:
union of kernel intervals / wall span of the timed region (approximated by the
last fraction of the trace)."""
import csv
import sys

rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(sys.argv[1]))))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
t0 = rows[0][0] + (rows[-1][1] - rows[0][0]) * (1 - frac)
iv = [(max(a, t0), b) for a, b in rows if b > t0]
busy, cur_s, cur_e = 0, None, None
for a, b in iv:
    if cur_e is None or a > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = a, b
    else:
        cur_e = max(cur_e, b)
busy += cur_e - cur_s
span = rows[-1][1] - t0
print(f"kernels {len(iv)}  busy {busy / span:.3f} of {span / 1e6:.2f} ms")
