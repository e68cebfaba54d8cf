#!/bin/bash
# Round-3 GPU session 2: attention A/B of the backward variants x per-kernel block orders (six shapes), the
# attention GPU tests over every variant, bench N=1, ResNet-50 kernel breakdown, world-4 one-GPU rehearsal.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 420 python -u scripts/bench_attn_ab.py --fwd 5 --bwd 3,9,10 --order=-2,0,2,3 --rounds 3 \
  > $OUT/r3_attn_ab2.jsonl 2> $OUT/r3_attn_ab2.err
rc=$?; echo "attn_ab rc=$rc"; tail -n 3 $OUT/r3_attn_ab2.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash_attn or hand_gemm_nt" -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/r3_pytest_attn.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -n 3 $OUT/r3_pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/r3_bench_n1_attn.json 2> $OUT/r3_bench_n1_attn.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/r3_bench_n1_attn.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/trace_resnet_kernels.py > $OUT/r3_resnet50_kernel_breakdown.jsonl 2> $OUT/r3_resnet50_kernel_breakdown.err
rc=$?; echo "resnet breakdown rc=$rc"; head -n 12 $OUT/r3_resnet50_kernel_breakdown.jsonl; tail -n 3 $OUT/r3_resnet50_kernel_breakdown.err
WORLDS="4" bash scripts/gpu_rehearsal.sh
exit $?
