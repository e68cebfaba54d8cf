#!/bin/bash
# Round 6 (r): the qkv narrow GEMM writing head-major for the window attention -- SwinIR A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_r
mkdir -p $OUT
for extra in "" "--precision fp32"; do
  for cfg in "PDT_HEAD_MAJOR_QKV=0" "PDT_HEAD_MAJOR_QKV=1"; do
    env $cfg timeout -k 10 300 python3 bench.py --workload swinir-stoke --loss feat --steps 20 --warmup 5 $extra > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
    echo "$cfg $extra: $(grep '^{' $OUT/b.log | tail -1 | cut -c1-160)" | tee -a $OUT/bench.txt
  done
done
PDT_HEAD_MAJOR_QKV=1 timeout -k 10 300 python3 bench.py --workload swinir-stoke --loss mse --steps 20 --warmup 5 > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
echo "mse: $(grep '^{' $OUT/b.log | tail -1 | cut -c1-160)" | tee -a $OUT/bench.txt
exit 0
