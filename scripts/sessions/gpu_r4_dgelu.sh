#!/bin/bash
# Round 4: fused MLP backward (c_proj dgrad + GELU backward + c_fc bias gradient in the hand GEMM's DGELU epilogue).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_dgelu${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  return $rc
}
MODE=check,bench ONLY=fc ROUNDS=3 run gemm 400 python -u scripts/bench_gemm_asm.py || exit $?
grep -E "dgelu|nt_fc\"|fullgrid" $OUT/gemm.log | cut -c1-260
run tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "fused or hand_gemm or gpt2" || exit $?
run bench 400 python bench.py --secondary 0 || exit $?
PDT_FUSED_DGELU=0 run bench_nodgelu 400 python bench.py --secondary 0 || exit $?
exit 0
