#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof stats.  Every GPU step has its
# own time limit; a crash/abort/timeout (exit >= 2 for pytest, != 0 otherwise)
# ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-10}
WARM=${WARM:-5}
echo "== env"; python -c "import torch; print(torch.__version__, torch.cuda.get_device_name(0))" || exit 1
echo "== lib identity"
timeout -k 10 120 python -c "
import torch, sys; sys.path.insert(0,'.')
import distributed_training_amd as D; D._lib.lib(); torch.zeros(1,device='cuda')
import collections
m=collections.OrderedDict()
for l in open('/proc/self/maps'):
    p=l.split()[-1]
    if 'amdhip64' in p or 'rccl' in p or 'gsync' in p: m[p]=1
print('\n'.join(m))" || exit 1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
  if [ $rc -ge 2 ]; then echo "pytest crashed/timed out: stopping"; exit $rc; fi
  echo "== smoke"
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  echo "== bench"
  timeout -k 10 600 python -u bench.py --gpus 1 --steps $STEPS --warmup $WARM ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if [ "${PROFILE:-0}" == "1" ]; then
  echo "== rocprofv3 kernel trace"
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 5 --warmup 3 --cpu-baseline 0 ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
  find $OUT/prof -name "*stats*" | head
fi
echo "== done"
