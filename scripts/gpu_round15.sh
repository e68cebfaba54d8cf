#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r15; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "conv3x3 or swinir" > $OUT/r15_pytest.log 2>&1 || { tail -60 $OUT/r15_pytest.log; exit 1; }
tail -2 $OUT/r15_pytest.log
timeout -k 10 120 python scripts/colsum_probe.py 2>&1 | grep '^{' || exit 1
for i in 1 2; do
echo "=== ours swinir $i"
timeout -k 10 400 python bench.py --workload swinir-stoke --steps 20 --warmup 5 2> $OUT/r15_a.err || exit $?
done
