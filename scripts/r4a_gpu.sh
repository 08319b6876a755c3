set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r4a; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread tests/test_clip_fold.py tests/test_zero_ds_step.py tests/test_gpu_native_hook.py tests/test_gpu_zero.py tests/test_gpu_zz_bench.py > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; echo "pytest rc=$rc"
[ $rc -ge 2 ] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 3000 $OUT/bench.json
