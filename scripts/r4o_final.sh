#!/bin/bash
# Round-4 final tree (after the bf16 -> bf16 pack's group of 4 and the unpack's
# fused reduction grid): bench.py --gpus 1, its rocprofv3 kernel trace + stats, and
# PMC traffic of the kernels those two changes touched (scripts/gpu_round.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 PROFILE=1 PMC=1 TAG=r4o PMC_OPS="resnet50:pack16b resnet50:unpacksq resnet50:unpack resnet50:sgd resnet152x2:unpacksq" \
  bash scripts/gpu_round.sh
