#!/bin/bash
# Round 5 (j): where the attention backward's per-workgroup fixed cost goes -- timing-only runs that skip the
# prologue loads / epilogue stores (PDT_FA_DIAG bits; results wrong) at the flagship shape.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_j${TAG:-}
mkdir -p $OUT
for v in 0 1 2 3 4 8 12 0; do
  echo "=== diag $v"
  PDT_FA_DIAG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/d$v -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/d$v.log 2>&1 || exit $?
done
exit 0
