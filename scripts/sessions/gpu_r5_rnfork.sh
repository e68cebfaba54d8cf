#!/bin/bash
# Round 5: ResNet-50 downsample-block fork (PDT_RESNET_FORK_DS) -- tests, then an interleaved bench A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_rnfork
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "resnet or conv or bn" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  echo "=== fork_ds $v"
  PDT_RESNET_FORK_DS=$v timeout -k 10 300 python3 bench.py --workload resnet50-ddp --steps 20 --warmup 5 > $OUT/bench$v.log 2>&1 || exit $?
  grep '^{' $OUT/bench$v.log | cut -c1-160
done
exit 0
