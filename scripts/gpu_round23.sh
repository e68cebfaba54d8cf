#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "attn or attention or causal or gpt2 or llama" > $OUT/r23_pytest.log 2>&1 || { tail -60 $OUT/r23_pytest.log; exit 1; }
tail -2 $OUT/r23_pytest.log
timeout -k 10 200 python scripts/attn_causal_probe.py 2>&1 | grep '^{' || exit 1
echo "=== flagship"
timeout -k 10 600 python bench.py 2> $OUT/r23_b.err || exit $?
