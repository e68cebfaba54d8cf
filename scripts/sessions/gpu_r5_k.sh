#!/bin/bash
# Round 5 (k): fused delta (dQ prologue loads O rows) vs the separate delta pass, per-kernel times.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_k${TAG:-}
mkdir -p $OUT
for v in 1 0 1 0; do
  echo "=== fuse $v"
  PDT_FA_FUSE_DELTA=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/f$v -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/f$v.log 2>&1 || exit $?
  grep '^{' $OUT/f$v.log
done
exit 0
