#!/bin/bash
# Round 5 (q): GEMM phase stamps for the plain / bias / GELU epilogues at c_fc, then a steady-state kernel trace of
# the flagship step (last 3 of 6 steps, marker = the optimizer kernel).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_q
mkdir -p $OUT
EPI_ONLY=1 timeout -k 10 150 python3 scripts/gemm_stamps.py > $OUT/stamps.log 2>&1 || exit $?
grep '^{' $OUT/stamps.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 3 --secondary 0 --overlap-probe 0 > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log | cut -c1-300
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_kernels.py "$f" --marker adamw_mt_kernel --last 3 --top 45 > $OUT/steady.txt && head -50 $OUT/steady.txt
rm -f "$f"
exit 0
