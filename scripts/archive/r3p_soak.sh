#!/bin/bash
# Long runs on the C++ hooks: ResNet-50 x256 for 300 timed steps, ResNet-18 x32 for 3000
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --gpus 1 --steps 300 --warmup 5 --cpu-baseline 0 --kernel-rates 0 > $OUT/r3p_soak_r50.json 2> $OUT/r3p_soak_r50.err || { tail $OUT/r3p_soak_r50.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 1 --model resnet18 --batch 32 --steps 3000 --warmup 5 --cpu-baseline 0 --kernel-rates 0 > $OUT/r3p_soak_r18.json 2> $OUT/r3p_soak_r18.err || { tail $OUT/r3p_soak_r18.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r3p_soak_r50.json", "gpurun_out/r3p_soak_r18.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), round(d["ms_per_step"], 3), d["parity"]["ok"], round(d["roofline"]["frac"], 3),
          d["memory"]["max_allocated_GB"])
PY
# probe: the Colossal fp16 CIFAR step as one hipGraph
timeout -k 10 300 python -u scripts/colossal_graph.py --steps 60 > $OUT/r3p_colossal_graph.jsonl 2> $OUT/r3p_colossal_graph.err || { tail -20 $OUT/r3p_colossal_graph.err; exit 1; }
cat $OUT/r3p_colossal_graph.jsonl
