#!/bin/bash
# Round-2 engine A/B on one GPU: parity of the kernels on both engines, then
# bench_kernels rows for the task engine (GS_ENGINE=0), the default split
# (streaming ops on the chunk-map engine) and everything on the chunk engine
# (254), plus chunk-ILP variants.  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r2a}
J=$OUT/${TAG}_kernels.jsonl
: > $J
echo "== kernel parity, default engines"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests_default.log 2>&1 || { tail -30 $OUT/${TAG}_tests_default.log; exit 1; }
tail -2 $OUT/${TAG}_tests_default.log
echo "== kernel parity, every op on the task engine"
GS_ENGINE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_tests_task.log 2>&1 || { tail -30 $OUT/${TAG}_tests_task.log; exit 1; }
tail -2 $OUT/${TAG}_tests_task.log
for round in 1 2; do
for m in "resnet50 1" "resnet152 2"; do
  set -- $m
  for eng in 0 254; do
    echo "== $1 x$2 GS_ENGINE=$eng (round $round)"
    GS_ENGINE=$eng timeout -k 10 300 python -u bench_kernels.py --model $1 --replicas $2 --skip-torch --iters 50 --tag eng$eng >> $J 2> $OUT/${TAG}_bk.err || { tail -20 $OUT/${TAG}_bk.err; exit 1; }
  done
  for v in ${VARIANTS:-g1 g2 g4}; do
    echo "== $1 x$2 variant $v GS_ENGINE=254 (round $round)"
    GS_ENGINE=254 GSYNC_LIB=distributed_training_amd/lib/variants/libgsync_$v.so timeout -k 10 300 python -u bench_kernels.py --model $1 --replicas $2 --skip-torch --iters 50 --tag ${v}_eng254 >> $J 2> $OUT/${TAG}_bk.err || { tail -20 $OUT/${TAG}_bk.err; exit 1; }
  done
done
done
python3 - "$J" <<'PY'
import json,sys,collections
rows=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]
d=collections.defaultdict(list)
for r in rows: d[(r['model'],r['replicas'],r['kernel'],r['tag'])].append(r['GBps'])
for k in sorted(d): print(k, ' '.join(f'{x:7.0f}' for x in d[k]))
PY
echo "== done"
