#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r21; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_llama -o l --output-format csv -- python3 bench.py --workload llama3-fsdp --steps 3 --warmup 1 > $OUT/prof_llama.log 2>&1 || exit $?
grep '"metric"' $OUT/prof_llama.log | cut -c1-200
