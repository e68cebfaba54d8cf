#!/bin/bash
# Round 4: flagship bench + its rocprofv3 kernel table (+ attention flagship timing).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_step${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log"
  return $rc
}
run attn 200 python -u scripts/bench_attn_flagship.py || exit $?
run bench 400 python bench.py --secondary 0 || exit $?
run rocprof 500 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --secondary 0 || exit $?
exit 0
