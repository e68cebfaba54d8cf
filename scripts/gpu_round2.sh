#!/bin/bash
# Leak test, micro-batch sweep, SwinIR Stoke workload, TunableOp GEMM search.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "future_leak or rope or llama" -p no:cacheprovider > $OUT/leak.log 2>&1; rc=$?
tail -n 12 $OUT/leak.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mb in 24 32; do
  echo "=== gpt2 mb$mb"
  timeout -k 10 300 python bench.py --micro-batch $mb --steps 6 --warmup 2 2> $OUT/mb$mb.err || exit $?
  tail -n 1 $OUT/mb$mb.err
done
echo "=== swinir"
timeout -k 10 300 python bench.py --workload swinir-stoke --steps 10 --warmup 3 2> $OUT/swinir.err || exit $?
tail -n 3 $OUT/swinir.err
echo "=== tunableop"
BENCH_ARGS="--micro-batch 16" TUNE_MS=30 bash scripts/tune_gemms.sh
