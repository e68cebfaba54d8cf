#!/bin/bash
# Round-3 closing check of HEAD on a fresh box: every pytest -m gpu test, smoke(), then the driver-style
# default bench (N=1).  Stops at the first failing GPU step.
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
run final_pytest_gpu 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
run final_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
run final_bench 500 python bench.py || exit $?
exit 0
