#!/bin/bash
# Round 5: the pruned engine (task engine and A/B-only knobs removed, raw Σg²
# partials for small plans) through the full GPU suite, then chunk-group sizes
# of the bucket and reduction kernels as library variants (lib/variants/<name>/,
# each with its own _gshook.so), interleaved over two rounds: the exposed tail's
# split, the kernel rows, configs[3]'s N=8-shard clip path.  One JSON line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5c; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  export GSYNC_TEST_PROGRESS_DIR=$OUT/progress
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -3 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  echo "smoke ok"
fi
VARIANTS="${VARIANTS:-gpack2 gpack4u4 gunpack1 gred4 gred8}" scripts/variant_rows.sh $OUT
