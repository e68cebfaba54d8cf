#!/bin/bash
# Round-6 full check: pytest -m gpu, smoke, default bench, rocprofv3 kernel stats of the
# flagship.  Stops at the first failing GPU step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_full${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  return $rc
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
run bench 500 python bench.py || exit $?
run rocprof 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 3 --warmup 3 --secondary 0 --overlap-probe 0 || exit $?
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_kernels.py "$f" --marker adamw_mt_kernel --last 3 --top 45 > $OUT/steady.txt && head -20 $OUT/steady.txt
rm -f "$f"
exit 0
