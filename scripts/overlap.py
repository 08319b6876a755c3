"""Overlap of libgsync's comm-stream work with the model's compute, from a
rocprofv3 --kernel-trace CSV.

    python scripts/overlap.py <kernel_trace.csv> [out.json]

For every kernel of the grad-sync path (libgsync pack/unpack on the comm
stream, RCCL kernels) the part of its [start, end) interval covered by
kernels of OTHER streams (MIOpen / ATen backward) counts as hidden; the
rest is exposed.  Reported per kernel class: launches, total µs, hidden µs,
hidden fraction.  The optimizer (launched on torch's stream after backward)
is reported as exposed by construction.
"""
import bisect
import csv
import json
import sys
from collections import defaultdict


def classify(name):
    n = name.lower()
    if "nccl" in n or "rccl" in n:
        return "rccl"
    if "gs::" in name:
        for k in ("PackOp", "UnpackOp", "SgdOp", "AdamOp", "SqnormOp", "UnscaleOp", "ScaleOp"):
            if k in name:
                return "gs_" + k
        return "gs_other"
    return None


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows]
    by_stream = defaultdict(list)
    for s, e, st, _ in ks:
        by_stream[st].append((s, e))
    merged = {}
    for st, iv in by_stream.items():  # union of each stream's busy intervals
        iv.sort()
        out = []
        for s, e in iv:
            if out and s <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([s, e])
        merged[st] = out

    def covered(s, e, own):
        tot = 0
        for st, iv in merged.items():
            if st == own:
                continue
            i = bisect.bisect_left(iv, [s, s]) - 1
            i = max(i, 0)
            while i < len(iv) and iv[i][0] < e:
                a, b = max(s, iv[i][0]), min(e, iv[i][1])
                if b > a:
                    tot += b - a
                i += 1
        return min(tot, e - s)

    agg = defaultdict(lambda: [0, 0, 0])
    for s, e, st, name in ks:
        c = classify(name)
        if c is None:
            continue
        a = agg[c]
        a[0] += 1
        a[1] += e - s
        a[2] += covered(s, e, st)
    res = {c: {"launches": n, "total_us": t / 1e3, "hidden_us": h / 1e3, "hidden_frac": h / t if t else None}
           for c, (n, t, h) in sorted(agg.items())}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
