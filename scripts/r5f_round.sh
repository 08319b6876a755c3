#!/bin/bash
# Round 5: the stream-packet probe with kernel-carried start events
# (scripts/micro/event_chain.hip), then scripts/r5b_round.sh on the current tree
# (GPU suite, smoke, the driver's bench, its rocprofv3 kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5f
timeout -k 10 90 scripts/micro/event_chain > gpurun_out/r5f/event_chain.jsonl 2> gpurun_out/r5f/event_chain.err || { cat gpurun_out/r5f/event_chain.err; exit 1; }
cat gpurun_out/r5f/event_chain.jsonl
TAG=r5f scripts/r5b_round.sh
