#!/bin/bash
# Round 6: PMC HBM traffic of every grad-sync kernel on the round's last tree
# (scripts/kernel_only.py under separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes,
# corrected by scripts/pmc_traffic.py as MI355X_MICROARCH.md's HBM section says),
# clip_grad_norm_'s scale pass (ClipScaleOp) among them.  Each pass under its own
# limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6i; mkdir -p $OUT
export TMPDIR=/tmp
for mo in resnet152x2:sgd resnet152x2:adam resnet50:sgd resnet50:adam resnet50:pack resnet50:unpack resnet50:sqnorm resnet50:sqpart resnet50:clipscale resnet50:clipsgd; do
  m=${mo%%:*}; o=${mo#*:}; reps=1; mm=$m
  case $m in *x2) mm=${m%x2}; reps=2;; esac
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch_${m}_$o -o k -- python3 scripts/kernel_only.py $mm 10 $o $reps >> $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write_${m}_$o -o k -- python3 scripts/kernel_only.py $mm 10 $o $reps >> $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
  python3 scripts/pmc_traffic.py $OUT/pmc_fetch_${m}_$o $OUT/pmc_write_${m}_$o $m/$o $OUT/pmc_traffic_r6i.json
  rm -rf $OUT/pmc_fetch_${m}_$o $OUT/pmc_write_${m}_$o
done
cat $OUT/pmc_traffic_r6i.json
echo done
