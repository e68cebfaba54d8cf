#!/bin/bash
# Round 6 (f): narrow-GEMM kernel (SwinIR linears) -- tests, microbench, SwinIR Stoke benches; then session e
# (micro-batch headroom, fake-world-8 rehearsal with real values, window-attention PMC).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "narrow or swinir or window_attention" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 scripts/bench_narrow.py > $OUT/bench_narrow.jsonl 2> $OUT/bench_narrow.err || { tail -20 $OUT/bench_narrow.err; exit 1; }
cat $OUT/bench_narrow.jsonl
run() {  # name, timeout, args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', d.get('value'), d.get('ms_per_step'), d.get('peak_mem_gb'))"
}
run swinir_feat_bf16 300 --workload swinir-stoke --loss feat --steps 10 --warmup 3 || exit 1
PDT_NARROW=0 run swinir_feat_bf16_nonarrow 300 --workload swinir-stoke --loss feat --steps 10 --warmup 3 || exit 1
run swinir_mse_bf16 300 --workload swinir-stoke --loss mse --steps 10 --warmup 3 || exit 1
bash scripts/sessions/gpu_r6_e.sh || exit 1
exit 0
