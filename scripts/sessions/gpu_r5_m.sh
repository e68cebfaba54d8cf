#!/bin/bash
# Round 5 (m): the persistent dK/dV kernel -- bitwise test against v3, then the flagship-shape attention bench
# v3 vs persistent (PDT_FA_DKDV) with per-kernel times.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_m${TAG:-}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "persistent_dkdv" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 3 4 3 4; do
  echo "=== dkdv $v"
  PDT_FA_DKDV=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/v$v -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/v$v.log 2>&1 || exit $?
  grep '^{' $OUT/v$v.log
done
exit 0
