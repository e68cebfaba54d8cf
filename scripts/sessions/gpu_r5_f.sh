#!/bin/bash
# Round 5 (f): ResNet-50 DDP parameter modes with single-process gradient stealing -- autocast over fp32 weights
# vs the bf16 compute copy (+ one multi-tensor gradient gather), interleaved; GPU tests of the DDP / ResNet paths.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_f${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep '^{' "$OUT/$name.log" | cut -c1-200; tail -n 1 "$OUT/$name.log" | cut -c1-200
  return $rc
}
run pytest_ddp 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "resnet or ddp or graph" || exit $?
run ac1_a 300 env PDT_RESNET_AUTOCAST=1 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run ac0_a 300 env PDT_RESNET_AUTOCAST=0 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run ac1_b 300 env PDT_RESNET_AUTOCAST=1 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run ac0_b 300 env PDT_RESNET_AUTOCAST=0 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run trace_ac0 300 env PDT_RESNET_AUTOCAST=0 python -u scripts/trace_resnet_kernels.py || exit $?
exit 0
