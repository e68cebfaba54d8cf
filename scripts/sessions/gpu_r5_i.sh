#!/bin/bash
# Round 5 (i): existing attention variants at the flagship shape after the scalar-addressing change:
# dQ v3 (4 waves, 2 workgroups / CU) vs v4 (8 waves, 1 / CU); forward v5 vs v7 / v8.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_i${TAG:-}
mkdir -p $OUT
for v in "PDT_FA_BWD=9" "PDT_FA_BWD=3" "PDT_FA_BWD=8" "PDT_FA_FWD=7" "PDT_FA_FWD=8" "PDT_FA_BWD=9"; do
  echo "=== $v"
  env $v timeout -k 10 200 python3 scripts/bench_attn_flagship.py > $OUT/v.log 2>&1 || exit $?
  grep '^{' $OUT/v.log
done
exit 0
