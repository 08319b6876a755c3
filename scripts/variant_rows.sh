#!/bin/bash
# Library variants of the engine (lib/variants/<name>/, each with its own
# _gshook.so) against the default, interleaved over two rounds: bench.py with
# the kernel rates (configs[3]'s N=8-shard clip path included), the exposed
# tail's split; one JSON line per run into <out>/rows.jsonl.
#   VARIANTS="a b c" [ENV_c="VAR=VALUE"] scripts/variant_rows.sh <out dir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in default $VARIANTS; do
    # a variant is a library build (lib/variants/<name>/) or, when ENV_<name> is set,
    # the default library under that VAR=VALUE environment setting
    envv=$(eval echo "\${ENV_$v:-}")
    if [ $v = default ] || [ -n "$envv" ]; then unset GSYNC_LIB; else export GSYNC_LIB=$PWD/distributed_training_amd/lib/variants/$v/libgsync.so; fi
    env $envv timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --zero-leg 0 --colossal-leg 0 --cpu-baseline 0 --parity 0 > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail -20 $OUT/b_${v}_$r.err; exit 1; }
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
