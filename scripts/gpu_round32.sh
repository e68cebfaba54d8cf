#!/bin/bash
# concurrent weight gradient on a side stream (PDT_WGRAD_STREAM=1) vs serial, flagship + Llama-3 8B
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
PDT_WGRAD_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "linear or gpt2 or llama" > $OUT/r32_pytest.log 2>&1 || { tail -60 $OUT/r32_pytest.log; exit 1; }
tail -2 $OUT/r32_pytest.log
for i in 1 2; do
echo "== serial $i"; timeout -k 10 600 python bench.py 2> $OUT/r32_a.err || exit $?
echo "== side stream $i"; PDT_WGRAD_STREAM=1 timeout -k 10 600 python bench.py 2> $OUT/r32_b.err || exit $?
done
echo "== llama serial"; timeout -k 10 600 python bench.py --workload llama3-fsdp --steps 5 --warmup 2 2> $OUT/r32_c.err || exit $?
echo "== llama side"; PDT_WGRAD_STREAM=1 timeout -k 10 600 python bench.py --workload llama3-fsdp --steps 5 --warmup 2 2> $OUT/r32_d.err || exit $?
