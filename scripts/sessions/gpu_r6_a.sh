#!/bin/bash
# Round 6 (a): steady-state kernel tables of the reference's own workload (SwinIR-S Stoke, feat_loss, bf16 and
# fp32) and of Llama-3 8B config 5, before this round's changes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_a
mkdir -p $OUT
trace() {  # name, timeout, bench args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 bench.py "$@" --overlap-probe 0 > $OUT/$name.log 2>&1 || return $?
  grep '^{' $OUT/$name.log | cut -c1-300
  local f=$(find $OUT/$name -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_kernels.py "$f" --marker adamw_mt_kernel --last 2 --top 45 > $OUT/${name}_steady.txt && head -30 $OUT/${name}_steady.txt
  rm -f "$f"
}
trace swinir_feat_bf16 300 --workload swinir-stoke --loss feat --steps 6 --warmup 3 || exit $?
trace swinir_feat_fp32 300 --workload swinir-stoke --loss feat --precision fp32 --steps 4 --warmup 2 || exit $?
trace llama3 500 --workload llama3-fsdp --steps 3 --warmup 2 || exit $?
exit 0
