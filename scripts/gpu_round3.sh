#!/bin/bash
# xGMI IPC collectives test, SwinIR kernel profile, TunableOp GEMM search (verbose so progress streams).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/xgmi_test.log 2>&1; rc=$?
tail -n 30 $OUT/xgmi_test.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "=== swinir profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_swinir -o swinir --output-format csv -- \
  python3 bench.py --workload swinir-stoke --steps 3 --warmup 1 > $OUT/prof_swinir.log 2>&1 || exit $?
tail -n 3 $OUT/prof_swinir.log
python3 scripts/trace_kernels.py $(find $OUT/prof_swinir -name "*kernel_trace.csv" | head -1) --top 40
echo "=== tunableop"
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_gfx950.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20
timeout -k 10 900 python bench.py --micro-batch 32 --steps 1 --warmup 1 > $OUT/tune_pass.log 2>&1 || exit $?
tail -n 2 $OUT/tune_pass.log
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 300 python bench.py --micro-batch 32 --steps 6 --warmup 2 2> $OUT/tuned.err || exit $?
tail -n 1 $OUT/tuned.err
PYTORCH_TUNABLEOP_ENABLED=0 timeout -k 10 300 python bench.py --micro-batch 32 --steps 6 --warmup 2 2> $OUT/untuned.err || exit $?
tail -n 1 $OUT/untuned.err
