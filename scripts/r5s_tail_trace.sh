#!/bin/bash
# Round 5: the end of backward in a DDP ResNet-50 step, kernel by kernel, under a
# rocprofv3 kernel trace (scripts/tail_trace.py): what the comm stream still runs
# when backward's last kernel ends.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/prof -o tail -- python3 -u scripts/tail_trace.py run > $OUT/run.log 2>&1 || { tail -30 $OUT/run.log; exit 1; }
python3 scripts/tail_trace.py analyze $(find $OUT/prof -name "*kernel_trace.csv" | head -1) > $OUT/tail.jsonl
head -1 $(find $OUT/prof -name "*kernel_trace.csv" | head -1) > $OUT/header.txt
rm -rf $OUT/prof
wc -l $OUT/tail.jsonl
