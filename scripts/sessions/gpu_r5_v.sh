#!/bin/bash
# Round 5 (v): LayerNorm forward grid cap (workgroups per CU) at the flagship shape; Llama residual-GEMM tests and
# config-5 A/B (PDT_RESID_GEMM 0 / 1).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_v
mkdir -p $OUT
for c in 16 4 8 32 96; do
  echo "=== cap $c"
  PDT_NORM_FWD_WG_PER_CU=$c timeout -k 10 200 python3 scripts/probe_gemm_residual_epilogue.py > $OUT/cap$c.log 2>&1 || exit $?
  grep '^{"shape' $OUT/cap$c.log | python3 -c "import sys,json; [print({k: v for k, v in json.loads(l).items() if k.startswith('ln') or k == 'shape'}) for l in sys.stdin]"
done
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "llama" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  echo "=== llama resid $v"
  PDT_RESID_GEMM=$v timeout -k 10 400 python3 bench.py --workload llama3-fsdp --steps 4 --warmup 2 --overlap-probe 0 > $OUT/llama$v.log 2>&1 || exit $?
  grep '^{' $OUT/llama$v.log | cut -c1-220
done
exit 0
