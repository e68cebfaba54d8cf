#!/bin/bash
# Round 5 (c): flash attention with scalar DMA addressing -- attention GPU tests, the flagship-shape attention
# bench, the default bench and the flagship kernel table.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_c${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400
  return $rc
}
run pytest_attn 500 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "flash or attn or llama or gpt2" || exit $?
run attn 300 python scripts/bench_attn_flagship.py || exit $?
run bench 500 python bench.py --secondary 0 || exit $?
run rocprof 500 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --secondary 0 || exit $?
exit 0
