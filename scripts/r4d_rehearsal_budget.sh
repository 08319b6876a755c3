#!/bin/bash
# The driver's N>1 command rehearsed at 4 ranks on the one GPU (gloo, ranks sharing
# the device: control flow, not a measurement), full ResNet-50 x 256, with a
# deliberately small --wall-budget-s: the headline, parity.ok, the legs that fit,
# and the skipped legs named in leg_errors.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4d; mkdir -p $OUT
BUDGET=${BUDGET:-240}
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 4 --pg-backend gloo --steps 5 --warmup 2 --wall-budget-s $BUDGET \
  > $OUT/n4_budget$BUDGET.json 2> $OUT/n4_budget$BUDGET.err
rc=$?; echo "rc=$rc"
tail -c 1500 $OUT/n4_budget$BUDGET.json
python3 - "$OUT/n4_budget$BUDGET.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", d["value"], "parity.ok", (d.get("parity") or {}).get("ok"), "leg_seconds", d.get("leg_seconds"))
print("leg_errors", d.get("leg_errors"), "warmup_s", d.get("warmup_s"))
PY
exit $rc
