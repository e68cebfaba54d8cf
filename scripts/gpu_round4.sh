#!/bin/bash
# SwinIR path: conv/norm/swinir tests, our vs stock SwinIR bench, SwinIR kernel profile.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "conv3x3 or swinir or layer_norm or rms_norm or fused_add_norm or window" -p no:cacheprovider > $OUT/r4_test.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" $OUT/r4_test.log | tail -n 40
tail -n 3 $OUT/r4_test.log
[ $rc -eq 0 ] || exit $rc
echo "=== swinir ours"
timeout -k 10 300 python bench.py --workload swinir-stoke --steps 10 --warmup 3 2> $OUT/swinir.err || exit $?
tail -n 2 $OUT/swinir.err
echo "=== swinir stock"
timeout -k 10 300 python scripts/bench_torch_baseline.py --workload swinir-stoke --steps 10 --warmup 3 2> $OUT/swinir_stock.err || exit $?
tail -n 2 $OUT/swinir_stock.err
echo "=== swinir profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_swinir2 -o swinir --output-format csv -- \
  python3 bench.py --workload swinir-stoke --steps 3 --warmup 1 > $OUT/prof_swinir2.log 2>&1 || exit $?
python3 scripts/trace_kernels.py $(find $OUT/prof_swinir2 -name "*kernel_trace.csv" | head -1) --top 30
