#!/bin/bash
# Round 6 tree check: the full GPU suite + smoke, the driver's default bench, and a
# rocprofv3 kernel trace of the same command (scripts/trace_bench.py -> the
# roofline's rocprof cross-check).  Each GPU step under its own limit; stop at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r6a}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  export GSYNC_TEST_PROGRESS_DIR=$OUT/progress
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -3 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  echo "smoke ok"
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = d["roofline"]
print("value", round(d["value"], 1), "ms", round(d["ms_per_step"], 3), "frac", round(r["frac"], 4), "in_step", round(r["in_step"]["frac"], 4) if "in_step" in r else None)
print("tail", d["grad_sync"].get("tail_ms"))
k = d.get("grad_sync_kernels") or {}
print("kernels", {n: round(v["frac"], 3) for n, v in k.get("kernels", {}).items()})
print("clip_zero", {n: (round(k[n]["avg_ms"] * 1e3, 1), round(k[n]["kernels_ms"] * 1e3, 1)) for n in ("clip_path_zero_n8", "clip_path_zero_n8_scalar") if n in k})
for n in ("zero2", "colossal"):
    z = d.get(n) or {}
    print(n, z.get("images_per_sec"), z.get("shard_update") or z.get("fused_adam"), (z.get("parity") or {}).get("ok"))
print("legs", d.get("leg_seconds"), d.get("leg_errors"), "parity", d["parity"]["ok"])
print("torch_ddp", d.get("torch_ddp"), "vs_baseline", d.get("vs_baseline"))
b = k.get("beyond_ic", {}).get("kernels", {})
print("beyond_ic", {n: (round(v["frac"], 3), round(v.get("frac_of_live_ceiling") or 0, 3)) for n, v in b.items()})
PY
if [ "${PROFILE:-1}" == "1" ]; then
  timeout -k 10 700 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python3 -u bench.py --cpu-baseline 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -20 $OUT/prof_bench.err; exit 1; }
  python3 scripts/trace_bench.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) 5 20 20 "$TAG" $OUT/trace_roofline.json
  for f in $(find $OUT/prof -name "*stats*.csv"); do cp $f $OUT/${TAG}_$(basename $f); done
  rm -rf $OUT/prof
fi
echo done
