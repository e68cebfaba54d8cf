#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_multiproc.py -x -v --timeout 120 --timeout-method thread \
  -k "syncbn or batchnorm or ddp" -p no:cacheprovider > $OUT/r8_test.log 2>&1; rc=$?
tail -n 2 $OUT/r8_test.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/r8_test.log | head; exit $rc; }
bash scripts/gpu_pmc.sh
