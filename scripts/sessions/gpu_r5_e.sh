#!/bin/bash
# Round 5 (e): A/B of the tuned-hipBLASLt arm of ops.linear.nt_matmul (PDT_NT_LT=auto vs 0) on the flagship,
# interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_e${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep '^{' "$OUT/$name.log" | cut -c1-200
  return $rc
}
run lt0_a 400 env PDT_NT_LT=0 python bench.py --secondary 0 || exit $?
run lt1_a 400 env PDT_NT_LT=auto python bench.py --secondary 0 || exit $?
run lt0_b 400 env PDT_NT_LT=0 python bench.py --secondary 0 || exit $?
run lt1_b 400 env PDT_NT_LT=auto python bench.py --secondary 0 || exit $?
exit 0
