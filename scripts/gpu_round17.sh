#!/bin/bash
# GPT-2 124M DDP kernel profile
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r17; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2s -o g --output-format csv -- python3 bench.py --workload gpt2-ddp --steps 6 --warmup 2 > $OUT/prof_gpt2s.log 2>&1 || exit $?
grep '"metric"' $OUT/prof_gpt2s.log | cut -c1-200
echo "=== flagship again (variance)"
timeout -k 10 600 python bench.py 2> $OUT/r17_flag.err || exit $?
