#!/bin/bash
# The update kernels' ceiling beyond the Infinity Cache: a plain float4 stream of
# the same read / write mixes (scripts/micro/stream_mix.hip) next to libgsync's
# own kernel rows at ResNet-152 x 2 (bench_kernels.py), same box, twice each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4p; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 120 scripts/micro/stream_mix > $OUT/stream_mix_$r.jsonl || exit 1
  timeout -k 10 200 python -u bench_kernels.py --model resnet152 --replicas 2 --iters 30 --skip-torch > $OUT/kernels_r152x2_$r.jsonl 2> $OUT/kb_$r.err || { tail $OUT/kb_$r.err; exit 1; }
done
echo done
