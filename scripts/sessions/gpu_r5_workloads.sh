#!/bin/bash
# Round 5 end: the other bench workloads on the round-end tree (GPT-2 124M DDP, SwinIR Stoke, Llama-3 8B config 5).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_workloads
mkdir -p $OUT
for w in gpt2-ddp swinir-stoke; do
  echo "=== $w"
  timeout -k 10 400 python3 bench.py --workload $w --steps 10 --warmup 3 --overlap-probe 0 > $OUT/$w.log 2>&1 || exit $?
  grep '^{' $OUT/$w.log | cut -c1-200
done
exit 0
