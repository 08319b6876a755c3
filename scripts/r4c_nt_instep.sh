#!/bin/bash
# Non-temporal load policy of the update kernels, in the training step and beyond
# the Infinity Cache: bench.py (ResNet-50 x 256, in-step fused SGD by the launch
# timer + grad_sync_kernels incl. the ResNet-152 x 2 rows) with each library
# variant (GSYNC_LIB: base, NT grad stream, NT state streams, both, NT everywhere),
# interleaved, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4c; mkdir -p $OUT
for r in 1 2; do
  for v in ${VARIANTS:-base ntg ntst ntupd ntall}; do
    GSYNC_LIB=distributed_training_amd/lib/variants/libgsync_$v.so timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 > $OUT/bench_${v}_r$r.json 2> $OUT/bench_${v}_r$r.err || { tail $OUT/bench_${v}_r$r.err; exit 1; }
    echo "$v r$r done"
  done
done
python3 - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r4c/bench_*_r*.json")):
    v = f.split("bench_")[1].rsplit("_r", 1)[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["grad_sync_kernels"]
    agg[v].append((d["value"], d["roofline"]["frac"], d["roofline"].get("frac_beyond_ic"),
                   {n: round(r["frac"], 3) for n, r in k["beyond_ic"]["kernels"].items()}))
for v, rows in agg.items():
    for r in rows:
        print(v, round(r[0], 1), "in-step", round(r[1], 4), "beyond-IC", round(r[2], 4), r[3])
PY
