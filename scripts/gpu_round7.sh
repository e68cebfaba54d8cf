#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_multiproc.py -x -v --timeout 120 --timeout-method thread \
  -k "batchnorm or resnet or syncbn or ddp" -p no:cacheprovider > $OUT/r7_test.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $OUT/r7_test.log | tail -n 40; tail -n 2 $OUT/r7_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/resnet_breakdown.py 2>&1 | grep -v amdgpu.ids || exit $?
echo "=== resnet50 bench"
timeout -k 10 300 python bench.py --workload resnet50-ddp --steps 10 --warmup 3 2> $OUT/r7_rn.err || exit $?
