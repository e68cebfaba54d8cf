#!/bin/bash
# Round 6 (p): window attention with chunked staging loads + fused relative-position table kernels.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_p
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "window or swinir or rel" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
true
for cfg in "PDT_SWIN_REL_TABLE_KERNELS=0" "PDT_SWIN_REL_TABLE_KERNELS=1"; do
  for extra in ""; do
    env $cfg timeout -k 10 300 python3 bench.py --workload swinir-stoke --loss feat --steps 20 --warmup 5 $extra > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
    echo "$cfg $extra: $(grep '^{' $OUT/b.log | tail -1 | cut -c1-160)" | tee -a $OUT/bench.txt
  done
done
exit 0
