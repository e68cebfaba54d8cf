#!/bin/bash
# Round-3 GPU session 3: persistent forward (v9) and the GQA-aware XCD grouping vs v5 on six shapes; attention
# GPU tests; ResNet-50 kernel breakdown (torch profiler); world-4 one-GPU rehearsal.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 420 python -u scripts/bench_attn_ab.py --fwd 5,9 --bwd=-1 --order=-2,0,1 --rounds 3 \
  > $OUT/r3_attn_ab3.jsonl 2> $OUT/r3_attn_ab3.err
rc=$?; echo "attn_ab rc=$rc"; tail -n 3 $OUT/r3_attn_ab3.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash_attn or hand_gemm_nt" -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/r3_pytest_attn.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -n 3 $OUT/r3_pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/trace_resnet_kernels.py > $OUT/r3_resnet50_kernel_breakdown.jsonl 2> $OUT/r3_resnet50_kernel_breakdown.err
rc=$?; echo "resnet breakdown rc=$rc"; head -n 14 $OUT/r3_resnet50_kernel_breakdown.jsonl; tail -n 3 $OUT/r3_resnet50_kernel_breakdown.err
[ $rc -eq 0 ] || exit $rc
WORLDS="4" bash scripts/gpu_rehearsal.sh
exit $?
