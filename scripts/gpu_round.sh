#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof stats, PMC traffic.  Every GPU
# step has its own time limit; a crash/abort/timeout ends the session.
#   env: SKIP_TESTS=1 SKIP_BENCH=1 PROFILE=1 PMC=1 STEPS WARM BENCH_ARGS PYTEST_ARGS TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
TAG=${TAG:-r1}
mkdir -p $OUT
STEPS=${STEPS:-20}
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
  timeout -k 10 900 python -u bench.py --gpus 1 --steps $STEPS --warmup $WARM ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
export TMPDIR=/tmp
if [ "${PROFILE:-0}" == "1" ]; then
  echo "== rocprofv3 kernel trace + stats (bench)"
  # the timed steps only after the warmup: no kernel-rate / parity launches in the trace
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o bench -- python3 -u bench.py --gpus 1 --steps $STEPS --warmup 3 --cpu-baseline 0 --kernel-rates 0 --parity 0 ${BENCH_ARGS:-} > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -20 $OUT/prof_$TAG.err; exit 1; }
  find $OUT/prof_$TAG -name "*stats*"
  python3 scripts/overlap.py $(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1) $OUT/overlap_$TAG.json > /dev/null || true
  python3 scripts/trace_roofline.py $(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1) $STEPS $OUT/trace_roofline_$TAG.json || true
  # keep the summaries (gpurun copies back <= 64 MiB): drop the full traces
  for f in $(find $OUT/prof_$TAG -name "*stats*.csv"); do cp $f $OUT/${TAG}_$(basename $f); done
  rm -rf $OUT/prof_$TAG
fi
if [ "${KBENCH:-0}" == "1" ]; then
  echo "== kernel microbench (bench_kernels, R50 and R152x2 > Infinity Cache)"
  timeout -k 10 300 python -u bench_kernels.py --model resnet50 --replicas 1 --iters 50 > $OUT/${TAG}_kernels_resnet50.jsonl 2> $OUT/${TAG}_kb.err || { tail $OUT/${TAG}_kb.err; exit 1; }
  timeout -k 10 300 python -u bench_kernels.py --model resnet152 --replicas 2 --iters 50 > $OUT/${TAG}_kernels_resnet152x2.jsonl 2>> $OUT/${TAG}_kb.err || { tail $OUT/${TAG}_kb.err; exit 1; }
fi
if [ "${PMC:-0}" == "1" ]; then
  echo "== PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes per kernel)"
  for mo in ${PMC_OPS:-resnet50:sgd resnet50:adam resnet50:pack resnet50:pack16 resnet50:unpack resnet50:sqnorm resnet50:unpacksq resnet152:sgd resnet152x2:pack resnet152x2:unpack resnet152x2:sqnorm}; do
    m=${mo%%:*}; o=${mo#*:}; reps=1; mm=$m
    case $m in *x2) mm=${m%x2}; reps=2;; esac
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch_${TAG}_${m}_$o -o k -- python3 scripts/kernel_only.py $mm 10 $o $reps >> $OUT/pmc_$TAG.log 2>&1 || { tail $OUT/pmc_$TAG.log; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write_${TAG}_${m}_$o -o k -- python3 scripts/kernel_only.py $mm 10 $o $reps >> $OUT/pmc_$TAG.log 2>&1 || { tail $OUT/pmc_$TAG.log; exit 1; }
    python3 scripts/pmc_traffic.py $OUT/pmc_fetch_${TAG}_${m}_$o $OUT/pmc_write_${TAG}_${m}_$o $m/$o $OUT/pmc_traffic_$TAG.json
    rm -rf $OUT/pmc_fetch_${TAG}_${m}_$o $OUT/pmc_write_${TAG}_${m}_$o
  done
fi
echo "== done"
