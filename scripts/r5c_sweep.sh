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
for r in 1 2; do
  for v in default ${VARIANTS:-gpack2 gpack4u4 gunpack1 gred4 gred8}; do
    if [ $v = default ]; then unset GSYNC_LIB; else export GSYNC_LIB=$PWD/distributed_training_amd/lib/variants/$v/libgsync.so; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --zero-leg 0 --colossal-leg 0 --cpu-baseline 0 --parity 0 > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail -20 $OUT/b_${v}_$r.err; exit 1; }
    python3 - "$OUT/b_${v}_$r.json" "$v" "$r" >> $OUT/rows.jsonl <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
k = d["grad_sync_kernels"]
t = d["grad_sync"]["tail_ms"]
row = {"variant": sys.argv[2], "round": int(sys.argv[3]), "images_per_sec": d["value"],
       "tail_total_us": t["total"] * 1e3, "tail_timed_us": t["total_timed_step"] * 1e3,
       "split_us": {x: round(t[x] * 1e3, 2) for x in ("queue", "pack", "collective", "unpack")},
       "r50": {n: round(v["frac"], 4) for n, v in k["kernels"].items()},
       "beyond_ic": {n: round(v["frac"], 4) for n, v in k["beyond_ic"]["kernels"].items()},
       "clip_zero_n8_us": {n: [round(k[n][f] * 1e3, 2) for f in ("avg_ms", "sqnorm_kernel_ms", "update_kernel_ms")]
                           for n in ("clip_path_zero_n8", "clip_path_zero_n8_scalar")},
       "hooks": d["config"].get("impl")}
print(json.dumps(row))
PY
    tail -1 $OUT/rows.jsonl
  done
done
unset GSYNC_LIB
echo done
