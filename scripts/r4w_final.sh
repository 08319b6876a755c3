#!/bin/bash
# Round-4 final tree (after the read-once NT rule for pack / unpack / Σg²): the
# driver's bench line + its rocprofv3 kernel trace first (fresh box, before any
# shared-GPU rehearsal writes MIOpen's find-db), PMC traffic of the pack and
# unpack, then the full -m gpu suite and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 PROFILE=1 PMC=1 TAG=r4w PMC_OPS="resnet152x2:pack resnet152x2:unpack resnet152x2:sqpart resnet50:unpack" \
  bash scripts/gpu_round.sh || exit $?
TAG=r4w bash scripts/gpu_tests.sh
