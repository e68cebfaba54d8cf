#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "conv3x3 or swinir" > $OUT/r27_pytest.log 2>&1 || { tail -60 $OUT/r27_pytest.log; exit 1; }
tail -2 $OUT/r27_pytest.log
for i in 1 2; do
echo "=== swinir $i"
timeout -k 10 400 python bench.py --workload swinir-stoke --steps 20 --warmup 5 2> $OUT/r27_a.err || exit $?
done
