#!/bin/bash
# Why is the whole-step hipGraph slower at ResNet-50 x256 (DESIGN §5 variants)?
# rocprofv3 kernel stats of the eager and the graph bench, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2graph; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --cpu-baseline 0 --kernel-rates 0 --parity 0 > /dev/null 2> $OUT/compile.err || exit 1
for g in 0 1; do
  d=$OUT/prof_g$g
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $d -o bench -- python3 -u bench.py --graph $g --steps 20 --warmup 3 --cpu-baseline 0 --kernel-rates 0 --parity 0 > $OUT/bench_g$g.json 2> $OUT/bench_g$g.err || { tail -5 $OUT/bench_g$g.err; exit 1; }
  s=$(find $d -name "*kernel_stats.csv" | head -1); cp "$s" $OUT/g${g}_kernel_stats.csv
  t=$(find $d -name "*kernel_trace.csv" | head -1); python3 scripts/busy.py "$t" > $OUT/g${g}_busy.txt 2>&1 || true
  rm -rf $d
  grep '^{' $OUT/bench_g$g.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph', $g, d['value'], d['ms_per_step'])"
done
