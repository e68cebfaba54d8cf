#!/bin/bash
# Round 6 (l): fp32 narrow GEMM / weight-gradient kernels (exact-f32 MFMA) -- tests, fp32 SwinIR bench + table.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "narrow or swinir" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() {  # name, timeout, args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', d.get('value'), d.get('ms_per_step'))"
}
run swinir_feat_fp32 300 --workload swinir-stoke --loss feat --precision fp32 --steps 8 --warmup 3 || exit 1
PDT_NARROW=0 run swinir_feat_fp32_nonarrow 300 --workload swinir-stoke --loss feat --precision fp32 --steps 8 --warmup 3 || exit 1
run swinir_feat_bf16 300 --workload swinir-stoke --loss feat --steps 10 --warmup 3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 bench.py --workload swinir-stoke --loss feat --precision fp32 --steps 4 --warmup 2 --overlap-probe 0 > $OUT/tr.log 2>&1 || exit 1
f=$(find $OUT/tr -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_kernels.py "$f" --marker adamw_mt_kernel --last 2 --top 50 > $OUT/swinir_fp32_steady.txt && head -30 $OUT/swinir_fp32_steady.txt | cut -c1-200
rm -f "$f"
exit 0
