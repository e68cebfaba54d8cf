#!/bin/bash
# fused window permutation: numerics + SwinIR end-to-end
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "window_perm or swinir or window_attention" > $OUT/r10_pytest.log 2>&1 || { tail -40 $OUT/r10_pytest.log; exit 1; }
tail -3 $OUT/r10_pytest.log
echo "=== ours swinir"
timeout -k 10 400 python bench.py --workload swinir-stoke --steps 20 --warmup 5 2> $OUT/r10_b.err || exit $?
