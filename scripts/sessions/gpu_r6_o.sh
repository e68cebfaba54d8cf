#!/bin/bash
# Round 6 (o): all kernels of the SwinIR bf16 step (after the fused L1), grouped by name prefix and grid.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_o
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 bench.py --workload swinir-stoke --loss feat --steps 4 --warmup 3 --overlap-probe 0 ${PREC_ARGS:-} > $OUT/tr.log 2>&1 || exit 1
f=$(find $OUT/tr -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_torch_kernels.py "$f" --match "" --top 60 --width 90 > $OUT/all_kernels.txt
python3 scripts/trace_torch_kernels.py "$f" --top 40 --width 300 > $OUT/torch_kernels.txt
rm -f "$f"
exit 0
