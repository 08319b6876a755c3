#!/bin/bash
# Round 5: do the exposed last bucket's grads keep their addresses across steps
# (scripts/grad_ptr_stability.py; a moved grad re-uploads the bucket's pointer
# table on the tail), and the PMC traffic of the headline kernel on this build
# (the fused SGD beyond the Infinity Cache and in the step's ResNet-50 size;
# separate FETCH_SIZE / WRITE_SIZE passes, scripts/kernel_only.py + pmc_traffic.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/grad_ptr_stability.py > $OUT/grad_ptrs.json 2> $OUT/grad_ptrs.err || { tail -20 $OUT/grad_ptrs.err; exit 1; }
cat $OUT/grad_ptrs.json
for mo in resnet152x2:sgd resnet50:sgd resnet50:sqnorm resnet50:sqpart; do
  m=${mo%%:*}; o=${mo#*:}; reps=1; mm=$m
  case $m in *x2) mm=${m%x2}; reps=2;; esac
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch_${m}_$o -o k -- python3 scripts/kernel_only.py $mm 10 $o $reps >> $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write_${m}_$o -o k -- python3 scripts/kernel_only.py $mm 10 $o $reps >> $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
  python3 scripts/pmc_traffic.py $OUT/pmc_fetch_${m}_$o $OUT/pmc_write_${m}_$o $m/$o $OUT/pmc_traffic_r5e.json
  rm -rf $OUT/pmc_fetch_${m}_$o $OUT/pmc_write_${m}_$o
done
cat $OUT/pmc_traffic_r5e.json
echo done
