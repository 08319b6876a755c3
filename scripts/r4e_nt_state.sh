#!/bin/bash
# The state-stream NT rule (gs_kernels.hip nt_state: p + fp32 states > 256 MiB ->
# non-temporal loads) checked in the training step where it flips: ResNet-50 Adam
# (307 MB of state) and ResNet-152 SGD (481 MB), GS_NT_STATE=0 (never) vs 2 (the
# rule), interleaved, 2 rounds; plus the default ResNet-50 SGD line (rule: normal
# loads, 204 MB) with every leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 400 python -u bench.py --gpus 1 --cpu-baseline 0 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
for r in 1 2; do
  for cfg in "adam:--optimizer adam" "r152:--model resnet152 --batch 128"; do
    n=${cfg%%:*}; a=${cfg#*:}
    for pol in 0 2; do
      GS_NT_STATE=$pol timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --kernel-rates 0 $a > $OUT/bench_${n}_nts${pol}_r$r.json 2> $OUT/bench_${n}_nts${pol}_r$r.err || { tail $OUT/bench_${n}_nts${pol}_r$r.err; exit 1; }
      echo "$n nts=$pol r$r done"
    done
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4e/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f.split("/")[-1], round(d["value"], 1), "in-step", round(r["frac"], 4), round(r["avg_launch_ms"] * 1e3, 1), "us",
          "beyond-IC", r.get("frac_beyond_ic"))
PY
