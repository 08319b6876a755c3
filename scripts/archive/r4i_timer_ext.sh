#!/bin/bash
# The plan launch timer on hipExtLaunchKernel's events (the kernel's own start / end)
# vs the two event packets around it (GS_TIMER_EXT=0), interleaved, 2 rounds each,
# against the rocprofv3 kernel trace of the same bench command; plus the GPU test
# modules of the kernels (after the engine moved into gs_engine.h + two TUs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_clip_fold.py tests/test_gpu_kernels.py \
  tests/test_zero_ds_step.py tests/test_gpu_large.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for ext in 1 0; do
    GS_TIMER_EXT=$ext timeout -k 10 400 python -u bench.py --gpus 1 --cpu-baseline 0 --parity 0 > $OUT/bench_ext${ext}_r$r.json 2> $OUT/bench_ext${ext}_r$r.err || { tail $OUT/bench_ext${ext}_r$r.err; exit 1; }
  done
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python3 -u bench.py --gpus 1 --steps 20 --warmup 3 --cpu-baseline 0 --parity 0 --kernel-rates 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 scripts/trace_roofline.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) 20 $OUT/trace_roofline_r4i.json || true
for f in $(find $OUT/prof -name "*stats*.csv"); do cp $f $OUT/r4i_$(basename $f); done
rm -rf $OUT/prof
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4i/bench_ext*.json")) + ["gpurun_out/r4i/prof_bench.json"]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]; k = (d["grad_sync_kernels"] or {}).get("kernels", {})
    print(f.split("/")[-1], round(d["value"], 1), "sgd", round(r["avg_launch_ms"] * 1e3, 2), "us frac", round(r["frac"], 4),
          "beyond", round(r.get("frac_beyond_ic") or 0, 4), {n: round(x["frac"], 3) for n, x in k.items()})
print(open("gpurun_out/r4i/trace_roofline_r4i.json").read())
PY
