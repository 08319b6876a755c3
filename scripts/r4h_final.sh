#!/bin/bash
# Round-4 final-tree measurements on one box: the descriptor-chain probe, then
# bench.py + its rocprofv3 kernel trace (the headline kernel's trace duration,
# profiles/trace_roofline.json) + PMC traffic passes of the grad-sync kernels that
# changed this round (scripts/gpu_round.sh SKIP_TESTS=1 PROFILE=1 PMC=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4h
timeout -k 10 120 scripts/micro/desc_chain > gpurun_out/r4h/desc_chain.jsonl || exit 1
SKIP_TESTS=1 PROFILE=1 PMC=1 TAG=r4h PMC_OPS="resnet50:sgd resnet50:adam resnet50:clipsgd resnet50:sqpart resnet152x2:sgd" \
  bash scripts/gpu_round.sh
