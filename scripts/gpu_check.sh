#!/bin/bash
# One GPU round trip: kernel/engine tests, smoke, short bench, rocprofv3 kernel stats.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1 from pytest).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 6 --warmup 2"}
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 $OUT/$name.log
  return $rc
}
python -c "import __graft_entry__ as g; g.build()" || exit 3
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 900 python bench.py $BENCH_ARGS || exit $?
if [ "${PROFILE:-1}" == "1" ]; then
  step rocprof 900 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --secondary 0 || exit $?
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
  python - <<'PY'
import csv, os
p = "gpurun_out/kernel_stats.csv"
if os.path.exists(p):
    rows = list(csv.DictReader(open(p)))
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in rows[:30]:
        print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}% n={r["Calls"]:>5} {r["Name"][:110]}')
PY
fi
exit 0
