#!/bin/bash
# Round 5: LayerNorm backward partial-row grid (PDT_NORM_BWD_WG 512 vs 256) on the whole flagship step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_lnbwd
mkdir -p $OUT
for v in 512 256 512 256; do
  echo "=== wg $v"
  PDT_NORM_BWD_WG=$v timeout -k 10 300 python3 bench.py --steps 6 --warmup 3 --secondary 0 --overlap-probe 0 > $OUT/bench$v.log 2>&1 || exit $?
  grep '^{' $OUT/bench$v.log | cut -c1-170
done
exit 0
