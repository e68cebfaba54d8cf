#!/bin/bash
# Round 5: GELU epilogue keeps gelu'(h) (not h); DGELU epilogue = multiply, round-0 derivative rows LDS-DMA'd under
# the main loop.  Tests at the production shape, GEMM A/B at c_fc / c_proj-dgrad, flagship with/without DGELU.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_dgelu${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  return $rc
}
run tests 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "hand_gemm or fused_linear or fused_gelu" || exit $?
MODE=check,bench ROUNDS=3 run gemm 500 python -u scripts/bench_gemm_asm.py || exit $?
grep -E "dgelu|nt_gelu|\"nt_|\"tt_" $OUT/gemm.log | cut -c1-300
PDT_FUSED_DGELU=1 run bench_dgelu 300 python bench.py --secondary 0 || exit $?
PDT_FUSED_DGELU=0 run bench_nodgelu 300 python bench.py --secondary 0 || exit $?
grep -h '"metric"' $OUT/bench_dgelu.log $OUT/bench_nodgelu.log | cut -c1-200
exit 0
