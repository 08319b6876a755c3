#!/bin/bash
# The driver's N>1 bench command rehearsed at 8 ranks: exactly
# `torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1
# --master-port P bench.py --gpus 8 --steps 20 --warmup 5`, with every default leg,
# plus --pg-backend gloo (the 8 ranks share the box's one GPU; RCCL refuses two ranks
# on a device) and a smaller batch (8 ResNet-50 activation sets on one GPU).  Not a
# measurement: the control flow, the legs' wall time at 8 ranks (the leg cost model's
# data), parity per leg and the exit status.  Every rank dumps its stacks each 60 s
# into the stderr file under gpurun_out/ (a slow compile is not silence).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r6n8}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp GSYNC_BENCH_TRACEBACK_S=60
timeout -k 10 ${LIMIT:-1100} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port ${PORT:-29611} bench.py --gpus 8 --steps 20 --warmup 5 --pg-backend gloo --batch ${BATCH:-64} \
  --wall-budget-s ${BUDGET:-900} ${BENCH_ARGS:-} > $OUT/n8_gloo.json 2> $OUT/n8_gloo.err
rc=$?
grep -v "^Thread\|^  File\|^Current thread\|^Timeout" $OUT/n8_gloo.err | grep "\[bench\]" | tail -30
echo "rc=$rc"
python3 - "$OUT/n8_gloo.json" <<'PY'
import json, sys
ls = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
if not ls:
    print("no line"); sys.exit(0)
d = ls[-1]
print("value", d["value"], "ms", d["ms_per_step"], "warmup_s", d.get("warmup_s"))
print("legs", d.get("leg_seconds"))
print("estimates", d.get("leg_estimates_s"))
print("errors", d.get("leg_errors"), "incomplete", d.get("legs_incomplete"))
print("parity", (d.get("parity") or {}).get("ok"))
for k in ("zero2", "colossal"):
    z = d.get(k) or {}
    print(k, z.get("images_per_sec"), (z.get("parity") or {}).get("ok"),
          ((z.get("overlap_allgather") or {}).get("parity") or {}).get("ok"))
ab = d.get("bucket_policy_ab") or {}
print("ab", ab.get("decision"), {n: (r.get("parity") or {}).get("ok") for n, r in (ab.get("variants") or {}).items()})
PY
exit $rc
