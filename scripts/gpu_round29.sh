#!/bin/bash
# sigmoid-form tanh-GELU: numerics tests, kernel microbench, dgrad layout variants, flagship bench
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "gelu or mlp or gpt2" > $OUT/r29_pytest.log 2>&1 || { tail -60 $OUT/r29_pytest.log; exit 1; }
tail -2 $OUT/r29_pytest.log
timeout -k 10 180 python -u scripts/bench_kernels.py --only gelu,adamw > $OUT/r29_kernels.jsonl 2> $OUT/r29_kernels.err || { tail $OUT/r29_kernels.err; exit 1; }
cat $OUT/r29_kernels.jsonl
timeout -k 10 180 python -u scripts/bench_gemm_roles.py dgrad > $OUT/r29_dgrad.jsonl 2> $OUT/r29_dgrad.err || { tail $OUT/r29_dgrad.err; exit 1; }
cat $OUT/r29_dgrad.jsonl
timeout -k 10 600 python bench.py 2> $OUT/r29_bench.err || exit $?
