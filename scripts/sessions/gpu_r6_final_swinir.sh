#!/bin/bash
# Round 6 final: SwinIR-S Stoke numbers (bf16 feat / MSE, fp32 feat) and the bf16 steady-state kernel table.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_final_swinir
mkdir -p $OUT
for args in "--loss feat" "--loss mse" "--loss feat --precision fp32"; do
  timeout -k 10 300 python3 bench.py --workload swinir-stoke $args --steps 20 --warmup 5 > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  grep '^{' $OUT/b.log | tail -1 >> $OUT/bench.jsonl
done
cat $OUT/bench.jsonl | cut -c1-150
bash scripts/sessions/gpu_r6_o.sh > /dev/null 2>&1 || exit 1
cp gpurun_out/r6_o/all_kernels.txt $OUT/all_kernels_bf16.txt
head -12 $OUT/all_kernels_bf16.txt | cut -c1-140
exit 0
