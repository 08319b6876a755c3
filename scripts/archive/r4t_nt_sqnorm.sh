#!/bin/bash
# Σg² non-temporal at every size (the new default): the driver's bench line first
# (fresh box, before anything else touches MIOpen's find-db), the clip-chain rows
# under the default, then the GPU modules on the Σg² / clip / ZeRO paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4t; mkdir -p $OUT
timeout -k 10 400 python -u bench.py --gpus 1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 200 python -u scripts/sqnorm_chain.py > $OUT/chain_default.jsonl 2> $OUT/chain.err || { tail $OUT/chain.err; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_clip_fold.py tests/test_zero_ds_step.py tests/test_gpu_zero.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r4t/bench.json").read().strip().splitlines()[-1])
k = d["grad_sync_kernels"]
print("value", round(d["value"], 1), "frac", round(d["roofline"]["frac"], 4), "beyond", round(d["roofline"]["frac_beyond_ic"], 4))
for name in ("sqnorm_f32", "sqnorm_partial_f32", "clip_path_sgd", "sgd_momentum_wd"):
    print(name, round(k["kernels"][name]["frac"], 4), round(k["beyond_ic"]["kernels"][name]["frac"], 4))
z = k["clip_path_zero_n8"]
print("zero_n8", round(z["avg_ms"] * 1e3, 1), "us kernels", round(z["kernels_ms"] * 1e3, 1), "vs scalar", round(z["vs_scalar_form"], 3))
for l in open("gpurun_out/r4t/chain_default.jsonl"):
    r = json.loads(l); print("chain", r["model"], r["replicas"], r["kernel"], round(r["frac"], 4))
PY
exit $rc
