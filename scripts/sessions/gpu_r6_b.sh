#!/bin/bash
# Round 6 (b): fp32 window attention on exact-f32 MFMA + fp32 window permutation + row-split norm backward:
# tests, then the fp32 SwinIR Stoke bench and the fp32 SwinIR / Llama-3 8B steady-state kernel tables.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "window_attention or window_perm or swinir or cross_entropy or norm" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_optim_cpu.py -m gpu > $OUT/pytest_optim.log 2>&1 || { tail -30 $OUT/pytest_optim.log; exit 1; }
tail -2 $OUT/pytest_optim.log
trace() {  # name, timeout, bench args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 bench.py "$@" --overlap-probe 0 > $OUT/$name.log 2>&1 || return $?
  grep '^{' $OUT/$name.log | cut -c1-300
  local f=$(find $OUT/$name -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_kernels.py "$f" --marker adamw_mt_kernel --last 2 --top 45 > $OUT/${name}_steady.txt && head -22 $OUT/${name}_steady.txt
  rm -f "$f"
}
timeout -k 10 300 python3 bench.py --workload swinir-stoke --loss feat --precision fp32 --steps 8 --warmup 3 > $OUT/bench_fp32.json 2> $OUT/bench_fp32.err || { tail -20 $OUT/bench_fp32.err; exit 1; }
cut -c1-300 $OUT/bench_fp32.json
trace swinir_feat_fp32 300 --workload swinir-stoke --loss feat --precision fp32 --steps 4 --warmup 2 || exit $?
trace llama3 500 --workload llama3-fsdp --steps 3 --warmup 2 || exit $?
exit 0
