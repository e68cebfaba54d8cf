#!/bin/bash
# Round 6 (c): window attention with next-window register prefetch and LDS-summed relative-bias gradient:
# window tests, SwinIR Stoke benches (bf16 feat / mse, fp32 feat) and the bf16 + fp32 steady-state kernel tables.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "window_attention or window_perm or swinir" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() {  # name, timeout, args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  cut -c1-200 $OUT/$name.json
}
run swinir_feat_bf16 300 --workload swinir-stoke --loss feat --steps 10 --warmup 3 || exit 1
run swinir_mse_bf16 300 --workload swinir-stoke --loss mse --steps 10 --warmup 3 || exit 1
run swinir_feat_fp32 300 --workload swinir-stoke --loss feat --precision fp32 --steps 8 --warmup 3 || exit 1
trace() {  # name, timeout, bench args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 bench.py "$@" --overlap-probe 0 > $OUT/$name.log 2>&1 || return $?
  local f=$(find $OUT/$name -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_kernels.py "$f" --marker adamw_mt_kernel --last 2 --top 45 > $OUT/${name}_steady.txt && head -16 $OUT/${name}_steady.txt
  rm -f "$f"
}
trace tr_swinir_feat_bf16 300 --workload swinir-stoke --loss feat --steps 5 --warmup 3 || exit $?
trace tr_swinir_feat_fp32 300 --workload swinir-stoke --loss feat --precision fp32 --steps 4 --warmup 2 || exit $?
exit 0
