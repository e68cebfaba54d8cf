#!/bin/bash
# colsum widths + rel-bias gather + window/swinir tests; SwinIR bench; GPT-2 1.3B FSDP micro-batch 48 trial
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r14; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "colsum or rel_bias or window or swinir or linear" > $OUT/r14_pytest.log 2>&1 || { tail -60 $OUT/r14_pytest.log; exit 1; }
tail -2 $OUT/r14_pytest.log
echo "=== ours swinir"
timeout -k 10 400 python bench.py --workload swinir-stoke --steps 20 --warmup 5 2> $OUT/r14_a.err || exit $?
echo "=== ours gpt2 1.3b mb48"
timeout -k 10 600 python bench.py --micro-batch 48 --steps 6 --warmup 2 2> $OUT/r14_b.err || exit $?
