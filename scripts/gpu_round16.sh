#!/bin/bash
# HIP-graph captured training step: numerics vs eager, then GPT-2 124M DDP eager vs graphed
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r16; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "graphed or adamw or fused_adam" > $OUT/r16_pytest.log 2>&1 || { tail -60 $OUT/r16_pytest.log; exit 1; }
tail -2 $OUT/r16_pytest.log
echo "=== gpt2-124m ddp eager"
timeout -k 10 300 python bench.py --workload gpt2-ddp --steps 20 --warmup 3 2> $OUT/r16_a.err || exit $?
echo "=== gpt2-124m ddp graph"
timeout -k 10 300 python bench.py --workload gpt2-ddp --steps 20 --warmup 3 --graph 1 2> $OUT/r16_b.err || { tail -20 $OUT/r16_b.err; exit 1; }
echo "=== gpt2-124m ddp mb4 eager (launch-bound regime)"
timeout -k 10 300 python bench.py --workload gpt2-ddp --micro-batch 4 --steps 20 --warmup 3 2> $OUT/r16_c.err || exit $?
echo "=== gpt2-124m ddp mb4 graph"
timeout -k 10 300 python bench.py --workload gpt2-ddp --micro-batch 4 --steps 20 --warmup 3 --graph 1 2> $OUT/r16_d.err || { tail -20 $OUT/r16_d.err; exit 1; }
