#!/bin/bash
# Round 5 (z): same-box A/B of the colsum(dO) stash (PDT_DX_COLSUM_STASH) and the fused CE forward+gradient
# (PDT_CE_FWD_GRAD) on the flagship bench.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_z
mkdir -p $OUT
for cfg in on off on off; do
  if [ $cfg = on ]; then export PDT_DX_COLSUM_STASH=1 PDT_CE_FWD_GRAD=1; else export PDT_DX_COLSUM_STASH=0 PDT_CE_FWD_GRAD=0; fi
  echo "=== $cfg"
  timeout -k 10 300 python3 bench.py --steps 6 --warmup 3 --secondary 0 --overlap-probe 0 > $OUT/bench_$cfg.log 2>&1 || exit $?
  grep '^{' $OUT/bench_$cfg.log | cut -c1-200
done
exit 0
