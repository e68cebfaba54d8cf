#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r24; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
echo "=== gpt2-124m ddp"
timeout -k 10 300 python bench.py --workload gpt2-ddp --steps 20 --warmup 3 2> $OUT/r24_a.err || exit $?
echo "=== llama3-8b fsdp"
timeout -k 10 600 python bench.py --workload llama3-fsdp --steps 4 --warmup 2 2> $OUT/r24_b.err || exit $?
echo "=== resnet50 ddp"
timeout -k 10 400 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 2> $OUT/r24_c.err || exit $?
echo "=== swinir"
timeout -k 10 400 python bench.py --workload swinir-stoke --steps 20 --warmup 5 2> $OUT/r24_d.err || exit $?
