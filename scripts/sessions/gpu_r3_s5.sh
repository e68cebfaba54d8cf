#!/bin/bash
# Round-3 session-4 follow-up: the new kernels' tests first (attention bias-gradient column sums, ragged-row
# weight gradient, fused add-norm with residual bias, hand NT GEMM incl. persistent), then the bench and a
# kernel-stats profile of the flagship.  Stops at the first failing GPU step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  return $rc
}
K=${K:-"bias_grad or ragged or fused_add_norm or hand_gemm or flash_attn or trainer_graph"}
run s5_pytest_new 600 python -u -m pytest ${FILES:-tests/test_kernels_gpu.py} -m gpu -q -x -k "$K" --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
run s5_bench 400 python bench.py --steps 10 --warmup 3 || exit $?
if [ "${PROFILE:-1}" == "1" ]; then
  mkdir -p $OUT/s5_prof
  run s5_prof 400 rocprofv3 --kernel-trace --stats -d $OUT/s5_prof -o flagship -- python3 bench.py --steps 3 --warmup 2 --secondary 0 || exit $?
  db=$(find $OUT/s5_prof -name "*.db" | head -n 1)
  python scripts/prof_db_stats.py "$db" --step-kernel adamw_mt_kernel --skip 2 --gaps 25 -o $OUT/s5_kernel_stats.csv > $OUT/s5_kernel_table.txt 2>&1 || true
  rm -f "$db"
  head -n 24 $OUT/s5_kernel_stats.csv | cut -c1-150
fi
exit 0
