#!/bin/bash
# Round 6 (s): 16-byte head-major stores in the narrow GEMM, wave-per-entry relative-bias scatter.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "window or swin or narrow or head_major or rel" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for extra in "" "--precision fp32"; do
  timeout -k 10 300 python3 bench.py --workload swinir-stoke --loss feat --steps 20 --warmup 5 $extra > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  echo "$extra: $(grep '^{' $OUT/b.log | tail -1 | cut -c1-160)" | tee -a $OUT/bench.txt
done
bash scripts/sessions/gpu_r6_o.sh > /dev/null 2>&1 || exit 1
head -25 gpurun_out/r6_o/all_kernels.txt | cut -c1-150
exit 0
