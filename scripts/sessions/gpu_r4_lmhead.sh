#!/bin/bash
# Round-4: tied LM-head weight gradient (no 3-stage program for many-tile TT outputs, 4 token slices), GEMM
# tests, flagship bench.
set -u
export PYTHONPATH=.
OUT=gpurun_out/r4_lm
mkdir -p $OUT
timeout -k 10 200 python -u scripts/bench_lm_head.py > $OUT/lm_head.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or linear or wgrad" -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log | cut -c1-200
