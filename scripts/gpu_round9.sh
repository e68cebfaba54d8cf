#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== stock gpt2-124m ddp"
timeout -k 10 300 python scripts/bench_torch_baseline.py --workload gpt2-ddp --steps 10 --warmup 3 2> $OUT/r9_a.err || exit $?
echo "=== ours gpt2-124m ddp"
timeout -k 10 300 python bench.py --workload gpt2-ddp --steps 10 --warmup 3 2> $OUT/r9_b.err || exit $?
echo "=== stock llama3-8b fsdp"
timeout -k 10 600 python scripts/bench_torch_baseline.py --workload llama3-fsdp --steps 4 --warmup 2 2> $OUT/r9_c.err || exit $?
tail -n 2 $OUT/r9_c.err
echo "=== ours llama3-8b fsdp"
timeout -k 10 600 python bench.py --workload llama3-fsdp --steps 4 --warmup 2 2> $OUT/r9_d.err || exit $?
