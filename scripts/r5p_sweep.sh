#!/bin/bash
# Round 5: Σg² with the combine as a second launch (GS_RED_FUSE=0) now that no
# event packet follows each launch (the round-2 choice of the in-kernel combine
# was measured with one), cached and with NT loads, against the default; two
# interleaved rounds.  scripts/micro/read_ceiling.hip put the plain read grid's
# reduction at 13.8 µs with NT loads (dependent scalar loads per iteration cost
# it 0.3 µs, profiles/r5/r5o_read_ceiling_tab.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5p; mkdir -p $OUT
export TMPDIR=/tmp
export ENV_fuse0="GS_RED_FUSE=0" ENV_fuse0nt="GS_RED_FUSE=0 GS_NT_SQNORM=1" ENV_nt="GS_NT_SQNORM=1"
VARIANTS="${VARIANTS:-fuse0 fuse0nt nt}" scripts/variant_rows.sh $OUT
for v in default fuse0 fuse0nt nt; do
  envv=$(eval echo "\${ENV_$v:-}")
  env $envv timeout -k 10 120 python -u scripts/sqnorm_shapes.py > $OUT/shapes_$v.jsonl 2> $OUT/shapes_$v.err || { tail -20 $OUT/shapes_$v.err; exit 1; }
done
echo done
