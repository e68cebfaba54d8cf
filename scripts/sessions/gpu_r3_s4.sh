#!/bin/bash
# Round-3 session-4 check after the container rebuild: pytest -m gpu, smoke, driver-style bench, the NT GEMM
# tile-boundary diagnostic and a kernel-stats profile of the flagship.  Stops at the first failing GPU step.
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
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  run s4_pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
  run s4_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
run s4_bench 400 python bench.py --steps 10 --warmup 3 || exit $?
[ "${DIAG:-0}" == "1" ] && { run s4_gemm_diag_nt 300 python -u scripts/bench_gemm_nt_diag.py || exit $?; }
if [ "${PROFILE:-1}" == "1" ]; then
  mkdir -p $OUT/s4_prof
  run s4_prof 400 rocprofv3 --kernel-trace --stats -d $OUT/s4_prof -o flagship -- python3 bench.py --steps 3 --warmup 2 --secondary 0 || exit $?
  db=$(find $OUT/s4_prof -name "*.db" | head -n 1)
  python scripts/prof_db_stats.py "$db" --step-kernel adamw_mt_kernel --skip 2 --gaps 25 -o $OUT/s4_kernel_stats.csv > $OUT/s4_kernel_table.txt 2>&1 || true
  rm -f "$db"
  head -n 30 $OUT/s4_kernel_stats.csv
fi
exit 0
