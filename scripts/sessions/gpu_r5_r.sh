#!/bin/bash
# Round 5 (r): unit-local item order of the persistent dK/dV kernel -- bitwise test against v3, then the
# flagship-shape attention bench with PDT_FA_DKDV_ORDER=0 (snake) vs default, per-kernel times.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_r${TAG:-}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "persistent_dkdv or persistent_dq or flagship_b96" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "=== order $v"
  if [ $v -eq 0 ]; then export PDT_FA_DKDV_ORDER=0; else unset PDT_FA_DKDV_ORDER; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/v$v -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/v$v.log 2>&1 || exit $?
  grep '^{' $OUT/v$v.log
  f=$(find $OUT/v$v -name "*kernel_stats.csv" | head -1); grep -o '"[^"]*fa_bwd_dkdv[^"]*",[0-9]*,[0-9]*,[0-9.]*' "$f" | cut -c1-20,80-
done
exit 0
