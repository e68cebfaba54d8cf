#!/bin/bash
# Round 5 (b): the attention k/v bias-gradient identities (dK/dV kernel without a column-sum epilogue), the
# two-level DGELU bias reduce and the 1-bit BatchNorm ReLU mask -- their GPU tests, the default bench (flagship +
# ResNet-50 secondary) and the flagship kernel table.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_b${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400
  return $rc
}
run pytest_sel 500 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "bias_grad or batchnorm or resnet or dgelu or flagship_b96 or colsum" || exit $?
run attn 300 python scripts/bench_attn_flagship.py || exit $?
run bench 500 python bench.py || exit $?
run rocprof 500 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 --secondary 0 || exit $?
exit 0
