#!/bin/bash
# MFMA window attention: tests, SwinIR bench + profile.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "window or swinir or tall_skinny or linear" -p no:cacheprovider > $OUT/r5_test.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" $OUT/r5_test.log | tail -n 40
tail -n 3 $OUT/r5_test.log
[ $rc -eq 0 ] || exit $rc
echo "=== swinir ours"
timeout -k 10 300 python bench.py --workload swinir-stoke --steps 10 --warmup 3 2> $OUT/swinir.err || exit $?
tail -n 2 $OUT/swinir.err
echo "=== swinir profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_swinir4 -o swinir --output-format csv -- \
  python3 bench.py --workload swinir-stoke --steps 3 --warmup 1 > $OUT/prof_swinir4.log 2>&1 || exit $?
python3 scripts/trace_kernels.py $(find $OUT/prof_swinir4 -name "*kernel_trace.csv" | head -1) --top 25
echo "=== gemm layouts"
timeout -k 10 300 python scripts/bench_gemm_layouts.py 2>&1 | tee $OUT/gemm_layouts.jsonl | grep -v amdgpu.ids
