#!/bin/bash
# Every bench.py workload of this framework on one MI355X (no stock-torch counterparts: those are in
# scripts/gpu_baselines.sh).  Each step has its own time limit; stops at the first failure.
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
run ours_gpt2_124m_ddp 300 python bench.py --workload gpt2-ddp --steps 10 --warmup 3 || exit $?
run ours_llama3_8b_fsdp 600 python bench.py --workload llama3-fsdp --act-ckpt 1 --act-ckpt-layers auto --steps 4 --warmup 2 || exit $?
run ours_swinir_feat_bf16 300 python bench.py --workload swinir-stoke --loss feat --steps 10 --warmup 3 || exit $?
run ours_swinir_mse_bf16 300 python bench.py --workload swinir-stoke --loss mse --steps 10 --warmup 3 || exit $?
run ours_swinir_feat_fp32 300 python bench.py --workload swinir-stoke --loss feat --precision fp32 --steps 6 --warmup 2 || exit $?
exit 0
