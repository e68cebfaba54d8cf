#!/bin/bash
# Round-5 Llama-3 8B config-5 check: selective activation recompute on every layer vs whole-layer recompute,
# micro-batch 8 and 16, then rocprofv3 kernel stats of the selective run.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_llama${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
  return $rc
}
run sel8 400 python bench.py --workload llama3-fsdp --steps 6 --warmup 2 --act-ckpt-policy selective || exit $?
run full8 400 python bench.py --workload llama3-fsdp --steps 6 --warmup 2 --act-ckpt-policy full || exit $?
run sel16 400 python bench.py --workload llama3-fsdp --steps 6 --warmup 2 --act-ckpt-policy selective --micro-batch 16 || exit $?
run rocprof 500 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o llama --output-format csv -- python bench.py --workload llama3-fsdp --steps 3 --warmup 1 --act-ckpt-policy selective || exit $?
exit 0
