#!/bin/bash
# Round 5 (u): residual adds in the projection GEMMs (PDT_RESID_GEMM) -- cost probe, numerics tests, flagship A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_u${TAG:-}
mkdir -p $OUT
timeout -k 10 200 python3 scripts/probe_gemm_residual_epilogue.py > $OUT/probe.log 2>&1 || exit $?
grep '^{' $OUT/probe.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "every_grad or linear_residual or fsdp_step_matches" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "=== resid $v"
  PDT_RESID_GEMM=$v timeout -k 10 300 python3 bench.py --steps 6 --warmup 3 --secondary 0 --overlap-probe 0 > $OUT/bench$v.log 2>&1 || exit $?
  grep '^{' $OUT/bench$v.log | cut -c1-200
done
exit 0
