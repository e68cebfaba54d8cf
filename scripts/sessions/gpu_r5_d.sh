#!/bin/bash
# Round 5 (d): ResNet-50 -- the NHWC max-pool kernels, fused BN stats/finalize and world-1 gradient stealing
# (tests), the DDP bench eager vs HIP-graph replay; the tuned-hipBLASLt NT arm (test + flagship bench).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_d${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  return $rc
}
run pytest_rn 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "maxpool or batchnorm or resnet or tuned_hipblaslt or ddp" || exit $?
run rn_eager 300 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run rn_graph 300 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 --resnet-graph 1 || exit $?
run rn_eager2 300 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run trace 300 python -u scripts/trace_resnet_kernels.py || exit $?
run flagship 500 python bench.py --secondary 0 || exit $?
exit 0
