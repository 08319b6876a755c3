#!/bin/bash
# The Σg² kernels' load policy where the clip path runs them (unpack -> Σg²
# partials -> clipped SGD, scripts/sqnorm_chain.py): GS_NT_SQNORM cached / NT /
# NT with the SGD's grad loads kept cached (GS_NT_SQ_HOT=1) / the size rule,
# interleaved, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4s; mkdir -p $OUT
for r in 1 2; do
  for pol in default 0 1 1hot; do
    unset GS_NT_SQ_HOT
    if [ $pol = default ]; then unset GS_NT_SQNORM; elif [ $pol = 1hot ]; then export GS_NT_SQNORM=1 GS_NT_SQ_HOT=1; else export GS_NT_SQNORM=$pol; fi
    timeout -k 10 200 python -u scripts/sqnorm_chain.py >> $OUT/chain.jsonl 2>> $OUT/chain.err || { tail $OUT/chain.err; exit 1; }
  done
done
unset GS_NT_SQNORM GS_NT_SQ_HOT
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/r4s/chain.jsonl"):
    r = json.loads(l)
    agg[(r["model"], r["replicas"], r["kernel"], r["GS_NT_SQNORM"])].append(round(r["frac"], 4))
for k in sorted(agg):
    print(k, agg[k])
PY
