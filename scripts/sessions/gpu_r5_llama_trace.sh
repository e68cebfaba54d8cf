#!/bin/bash
# Round 5: steady-state kernel table of the Llama-3 8B config-5 step (FSDP + selective recompute on all layers).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_llama_trace
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload llama3-fsdp --steps 3 --warmup 2 --overlap-probe 0 > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log | cut -c1-250
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_kernels.py "$f" --marker adamw_mt_kernel --last 2 --top 40 > $OUT/steady.txt && head -42 $OUT/steady.txt
rm -f "$f"
exit 0
