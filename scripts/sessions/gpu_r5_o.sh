#!/bin/bash
# Round 5 (o): persistent dQ kernel -- test against the per-item dQ kernel, then the flagship-shape attention bench
# (PDT_FA_DQP=1 persistent vs 0) with per-kernel times.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_o${TAG:-}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "persistent_dq or persistent_dkdv or bias_grad or flagship_b96 or full_grid" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "=== dqp $v"
  PDT_FA_DQP=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/v$v -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/v$v.log 2>&1 || exit $?
  grep '^{' $OUT/v$v.log
done
exit 0
