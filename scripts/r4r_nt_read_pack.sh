#!/bin/bash
# GS_NT_READ_ONCE A/B after the rule reached the pack and unpack (never / always /
# beyond the cache = default): Σg², partials, clip path, SGD, pack, unpack,
# interleaved, 2 rounds (scripts/nt_read_sweep.py); then the kernel / clip / DDP
# GPU tests on the new rule.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4r; mkdir -p $OUT
for r in 1 2; do
  for pol in default 0 1; do
    if [ $pol = default ]; then unset GS_NT_READ_ONCE; else export GS_NT_READ_ONCE=$pol; fi
    timeout -k 10 200 python -u scripts/nt_read_sweep.py >> $OUT/nt_read.jsonl 2>> $OUT/nt_read.err || { tail $OUT/nt_read.err; exit 1; }
  done
done
unset GS_NT_READ_ONCE
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4r/nt_read.jsonl"):
    r = json.loads(l)
    agg[(r["model"], r["replicas"], r["kernel"], r["GS_NT_READ_ONCE"])].append(round(r["frac"], 4))
for k in sorted(agg):
    print(k, agg[k])
PY
timeout -k 10 300 python -u -m pytest tests/test_clip_fold.py tests/test_gpu_kernels.py tests/test_gpu_large.py tests/test_gpu_ddp.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; exit $rc
