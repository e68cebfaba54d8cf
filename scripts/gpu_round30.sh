#!/bin/bash
# transposed-layout data gradients: tests, GEMM role microbench, flagship + Llama-3 8B + GPT-2 124M benches
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "transpose or linear or gpt2 or llama" > $OUT/r30_pytest.log 2>&1 || { tail -60 $OUT/r30_pytest.log; exit 1; }
tail -2 $OUT/r30_pytest.log
timeout -k 10 180 python -u scripts/bench_gemm_roles.py dgrad > $OUT/r30_dgrad.jsonl 2> $OUT/r30_dgrad.err || { tail $OUT/r30_dgrad.err; exit 1; }
cat $OUT/r30_dgrad.jsonl
timeout -k 10 600 python bench.py 2> $OUT/r30_bench.err || exit $?
timeout -k 10 600 python bench.py 2> $OUT/r30_bench2.err || exit $?
timeout -k 10 600 python bench.py --workload llama3-fsdp --steps 5 --warmup 2 2> $OUT/r30_llama.err || exit $?
timeout -k 10 600 python bench.py --workload gpt2-ddp 2> $OUT/r30_gpt2s.err || exit $?
