#!/bin/bash
# VERDICT r3's per_wg candidate for the updates: GS_UPD_CONTIG 0 (one group per
# workgroup, the default) / 1024 / 2048 / 4096 / 8192 contiguous-range grids,
# SGD and Adam at ResNet-50 and ResNet-152 x 2 (scripts/update_rows.py),
# interleaved, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4y; mkdir -p $OUT
for r in 1 2; do
  for c in 0 1024 2048 4096 8192; do
    GS_UPD_CONTIG=$c timeout -k 10 200 python -u scripts/update_rows.py >> $OUT/rows.jsonl 2>> $OUT/rows.err || { tail $OUT/rows.err; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4y/rows.jsonl"):
    r = json.loads(l)
    agg[(r["set"], r["kernel"], int(r["GS_UPD_CONTIG"]))].append(round(r["frac"], 4))
for k in sorted(agg):
    print(k, agg[k])
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sgd or adam" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; exit $rc
