#!/bin/bash
# Round 5 (h): per-kernel attention times at S = 1k vs 8k (same tokens) under rocprofv3 kernel stats.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_h${TAG:-}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p1k -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/p1k.log 2>&1 || exit $?
B=12 S=8192 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p8k -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/p8k.log 2>&1 || exit $?
exit 0
