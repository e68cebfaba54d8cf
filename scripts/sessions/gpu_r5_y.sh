#!/bin/bash
# Round 5 (y): fused CE forward + gradient, the colsum(dO) stash fix -- GPU suite, then the flagship A/B
# (PDT_CE_FWD_GRAD 0 / 1) with a steady-state kernel table of the default.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_y
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "=== ce_fwd_grad $v"
  PDT_CE_FWD_GRAD=$v timeout -k 10 300 python3 bench.py --steps 6 --warmup 3 --secondary 0 --overlap-probe 0 > $OUT/bench$v.log 2>&1 || exit $?
  grep '^{' $OUT/bench$v.log | cut -c1-200
done
exit 0
