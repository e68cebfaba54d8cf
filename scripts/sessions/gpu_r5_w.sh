#!/bin/bash
# Round 5 (w): LayerNorm backward partial-row grid (PDT_NORM_BWD_WG) at the flagship shape.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_w2
mkdir -p $OUT
for c in 512 256 128 384 256 512 128; do
  PDT_NORM_BWD_WG=$c timeout -k 10 120 python3 scripts/probe_norm_bwd.py > $OUT/bwd$c.log 2>&1 || exit $?
  grep '^{' $OUT/bwd$c.log
done
exit 0
