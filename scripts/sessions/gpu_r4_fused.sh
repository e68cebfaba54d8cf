#!/bin/bash
# Round 4: fused c_fc + bias + GELU on the hand GEMM -- GEMM / fused tests, then the flagship bench (A/B with
# PDT_FUSED_GELU=0) and its kernel table.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_fused${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  return $rc
}
run tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "fused_linear or hand_gemm or wgrad or gpt2" || exit $?
run bench 400 python bench.py --secondary 0 || exit $?
PDT_FUSED_GELU=0 run bench_unfused 400 python bench.py --secondary 0 || exit $?
run rocprof 500 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --secondary 0 || exit $?
exit 0
