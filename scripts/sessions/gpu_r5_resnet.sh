#!/bin/bash
# Round 5: ResNet-50 DDP secondary -- bench both parameter modes (autocast over fp32 weights vs the bf16 compute
# copy), then the in-process kernel breakdown of each (torch profiler; rocprofv3 makes MIOpen fall back).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_resnet${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  return $rc
}
run bench_ac1 300 env PDT_RESNET_AUTOCAST=1 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run bench_ac0 300 env PDT_RESNET_AUTOCAST=0 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 || exit $?
run trace_ac1 300 env PDT_RESNET_AUTOCAST=1 python -u scripts/trace_resnet_kernels.py || exit $?
run trace_ac0 300 env PDT_RESNET_AUTOCAST=0 python -u scripts/trace_resnet_kernels.py || exit $?
exit 0
