#!/bin/bash
# Round 6 (k): SwinIR bf16 grid A/B -- narrow-row norm backward workgroups (512 / 1024 / 2048) and fused-MLP
# backward workgroups (256 / 512 / 768).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_k
mkdir -p $OUT
run() {  # name, timeout, args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', d.get('value'), d.get('ms_per_step'))"
}
A="--workload swinir-stoke --loss feat --steps 12 --warmup 3"
run base 300 $A || exit 1
PDT_NORM_SMALL_BWD_WG=1024 run norm1024 300 $A || exit 1
PDT_NORM_SMALL_BWD_WG=2048 run norm2048 300 $A || exit 1
PDT_SWIN_MLP_BWD_WG=512 run mlp512 300 $A || exit 1
PDT_SWIN_MLP_BWD_WG=768 run mlp768 300 $A || exit 1
run base2 300 $A || exit 1
exit 0
