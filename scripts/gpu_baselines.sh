#!/bin/bash
# One GPU round trip measuring every BASELINE.json workload on 1 MI355X: our stack vs stock PyTorch-ROCm.
# Each step has its own time limit; the script stops at the first failure.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 $to "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  echo "rc=$rc"; tail -n 2 $OUT/$name.err; cat $OUT/$name.json
  return $rc
}
run ours_gpt2_1.3b_fsdp 300 python bench.py --steps 8 --warmup 3 || exit $?
run torch_gpt2_1.3b_fsdp 300 python scripts/bench_torch_baseline.py --workload gpt2-fsdp --steps 8 --warmup 3 || exit $?
run ours_resnet50_ddp 300 python bench.py --workload resnet50-ddp --steps 10 --warmup 3 || exit $?
run torch_resnet50_ddp 300 python scripts/bench_torch_baseline.py --workload resnet50-ddp --steps 10 --warmup 3 || exit $?
run ours_gpt2_124m_ddp 300 python bench.py --workload gpt2-ddp --steps 10 --warmup 3 || exit $?
run ours_llama3_8b_fsdp 600 python bench.py --workload llama3-fsdp --steps 4 --warmup 2 || exit $?
exit 0
