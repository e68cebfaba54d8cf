#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "linear or gpt2" > $OUT/r20_pytest.log 2>&1 || { tail -60 $OUT/r20_pytest.log; exit 1; }
tail -2 $OUT/r20_pytest.log
for i in 1 2; do
echo "=== flagship $i"
timeout -k 10 600 python bench.py 2> $OUT/r20_b.err || exit $?
done
echo "=== flagship no layout tune"
PDT_WGRAD_TUNE=0 timeout -k 10 600 python bench.py 2> $OUT/r20_c.err || exit $?
