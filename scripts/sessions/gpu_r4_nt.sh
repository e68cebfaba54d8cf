#!/bin/bash
# Round 4: flagship with the per-shape hand-NT-vs-hipBLASLt choice (A/B against PDT_NT_HIP=0) + GEMM tests.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_nt${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-250
  return $rc
}
run tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or wgrad or fused or gpt2 or linear" || exit $?
run bench 400 python bench.py --secondary 0 || exit $?
PDT_NT_HIP=0 run bench_lt 400 python bench.py --secondary 0 || exit $?
run bench2 400 python bench.py --secondary 0 || exit $?
exit 0
