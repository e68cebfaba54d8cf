#!/bin/bash
# Round 5 (l): backward block order -- heavy-first (default) vs the cycled order (PDT_FA_CYCLE bits 2 dK/dV,
# 4 dQ) that staggers the workgroups' HBM-bound prologues.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_l${TAG:-}
mkdir -p $OUT
for v in 0 2 4 6 0 6; do
  echo "=== cycle $v"
  PDT_FA_CYCLE=$v timeout -k 10 120 python3 scripts/bench_attn_flagship.py > $OUT/c$v.log 2>&1 || exit $?
  grep '^{' $OUT/c$v.log
done
exit 0
