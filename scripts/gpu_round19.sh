#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "linear or gpt2 or graphed or causal" > $OUT/r19_pytest.log 2>&1 || { tail -60 $OUT/r19_pytest.log; exit 1; }
tail -2 $OUT/r19_pytest.log
echo "=== gpt2-124m ddp"
timeout -k 10 300 python bench.py --workload gpt2-ddp --steps 20 --warmup 3 2> $OUT/r19_a.err || exit $?
echo "=== flagship"
timeout -k 10 600 python bench.py 2> $OUT/r19_b.err || exit $?
