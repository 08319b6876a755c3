#!/bin/bash
# Round 6: configs[3] standalone on both engines, 20 timed steps after 5 warm-up steps each:
# torch FSDP(SHARD_GRAD_OP, bf16 MixedPrecision) + clip + fused AdamW (bench.py --impl torch
# --engine zero2) and libgsync ZeRO-2 (--engine zero2) — the check behind the zero2 leg's
# same-run torch comparison.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r6e
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --impl torch --engine zero2 --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r6e/torch_zero2.json 2> gpurun_out/r6e/torch_zero2.err && \
timeout -k 10 400 python -u bench.py --engine zero2 --steps 20 --warmup 5 --cpu-baseline 0 --kernel-rates 0 > gpurun_out/r6e/gsync_zero2.json 2> gpurun_out/r6e/gsync_zero2.err
rc=$?
python3 - <<'PY'
import json
for f in ("torch_zero2", "gsync_zero2"):
    try:
        d = [json.loads(l) for l in open(f"gpurun_out/r6e/{f}.json") if l.startswith("{")][-1]
        print(f, round(d["value"], 1), round(d["ms_per_step"], 2))
    except Exception as e:
        print(f, "no line", e)
PY
exit $rc
