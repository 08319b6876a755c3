#!/bin/bash
# Round-3 measurements: eager CIFAR step host breakdown (C++ vs Python hooks,
# torch DDP), and grad-sync kernel rates of library variants (bf16 pack group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u scripts/cifar_host.py --steps 100 --out $OUT/r3d_cifar_host.jsonl > $OUT/r3d_cifar.log 2>&1 || { tail -20 $OUT/r3d_cifar.log; exit 1; }
GSYNC_NATIVE_HOOK=0 timeout -k 10 300 python -u scripts/cifar_host.py --steps 100 --impls gsync --out $OUT/r3d_cifar_host_pyhook.jsonl >> $OUT/r3d_cifar.log 2>&1 || { tail -20 $OUT/r3d_cifar.log; exit 1; }
cat $OUT/r3d_cifar_host.jsonl $OUT/r3d_cifar_host_pyhook.jsonl
for r in 1 2; do
  for v in libgsync variants/libgsync_p16g1 variants/libgsync_p16g4 variants/libgsync_p16g8; do
    GSYNC_LIB=distributed_training_amd/lib/$v.so timeout -k 10 200 python -u scripts/kernel_rates.py resnet50 $(basename $v) >> $OUT/r3d_kernel_rates.jsonl 2>> $OUT/r3d_kr.err || { tail $OUT/r3d_kr.err; exit 1; }
  done
done
cat $OUT/r3d_kernel_rates.jsonl
# GPU busy fraction of the eager CIFAR step with the C++ hooks (kernel trace of one gsync round)
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/r3d_prof_cifar -o cifar -- python3 -u scripts/cifar_host.py --steps 200 --impls gsync --rounds 1 > $OUT/r3d_cifar_prof.log 2>&1 || { tail $OUT/r3d_cifar_prof.log; exit 1; }
python3 scripts/busy.py $(find $OUT/r3d_prof_cifar -name "*kernel_trace.csv" | head -1) 0.3 | tee $OUT/r3d_cifar_busy.txt
rm -rf $OUT/r3d_prof_cifar
