#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_rn50 -o rn50 --output-format csv -- python3 bench.py --workload resnet50-ddp --steps 3 --warmup 2 > $OUT/prof_rn50.log 2>&1 || exit $?
tail -n 1 $OUT/prof_rn50.log
python3 scripts/trace_kernels.py $(find $OUT/prof_rn50 -name "*kernel_trace.csv" | head -1) --top 40
