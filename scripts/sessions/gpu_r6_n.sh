#!/bin/bash
# Round 6 (n): fused L1 loss + accumulating DDP gradient gather -- tests, then SwinIR bf16 / fp32 A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_n
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "l1 or multi_tensor or steal_acc or swinir or window or narrow" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for cfg in "PDT_FUSED_L1=1"; do
  for extra in "" "--precision fp32"; do
    env $cfg timeout -k 10 300 python3 bench.py --workload swinir-stoke --loss feat --steps 20 --warmup 5 $extra > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
    echo "$cfg $extra: $(grep '^{' $OUT/b.log | tail -1 | cut -c1-160)"
  done
done
exit 0
