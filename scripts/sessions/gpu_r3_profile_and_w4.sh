#!/bin/bash
# Round-3 GPU session: attention A/B (new 8-wave kernels, XCD-grouped block order), flagship kernel-stats
# profile, xGMI timeout diagnosis test, world-4 one-GPU rehearsal (default and 2 hardware queues per rank).
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT/prof_r3
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = attn ]; then
  timeout -k 10 420 python -u scripts/bench_attn_ab.py --shapes gpt2-1.3b-b96,gpt2-1.3b,gpt2-1.3b-full,long-4k \
    --fwd 5,7,8 --bwd 3,8,9 --order 0,1 --rounds 3 > $OUT/r3_attn_ab.jsonl 2> $OUT/r3_attn_ab.err
  rc=$?; echo "attn_ab rc=$rc"; tail -3 $OUT/r3_attn_ab.err; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r3 -o flagship -- python3 bench.py --steps 3 --warmup 2 --secondary 0 > $OUT/r3_prof_flagship.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -2 $OUT/r3_prof_flagship.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = w4 ]; then
  timeout -k 10 200 python -u -m pytest tests/test_xgmi_gpu.py -k timeout -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r3_xgmi_timeout_test.log 2>&1
  rc=$?; echo "timeout test rc=$rc"; tail -2 $OUT/r3_xgmi_timeout_test.log; [ $rc -eq 0 ] || exit $rc
  PDT_XGMI_TIMEOUT_S=20 PDT_BENCH_BACKEND=gloo PDT_XGMI=1 timeout -k 10 240 python bench.py --gpus 4 --micro-batch 2 --steps 3 --warmup 1 --secondary 0 > $OUT/rehearsal_gpt2_fsdp_w4_q4.log 2>&1
  rc=$?
  echo "w4 default queues rc=$rc"; grep -h "timed out" $OUT/rehearsal_gpt2_fsdp_w4_q4.log | head -4; tail -2 $OUT/rehearsal_gpt2_fsdp_w4_q4.log
  [ $rc -eq 0 ] && exit 0
  [ $rc -eq 1 ] || exit $rc
  GPU_MAX_HW_QUEUES=2 PDT_XGMI_TIMEOUT_S=20 PDT_BENCH_BACKEND=gloo PDT_XGMI=1 timeout -k 10 240 python bench.py --gpus 4 --micro-batch 2 --steps 3 --warmup 1 --secondary 0 > $OUT/rehearsal_gpt2_fsdp_w4_q2.log 2>&1
  rc=$?
  echo "w4 2 queues rc=$rc"; grep -h "timed out" $OUT/rehearsal_gpt2_fsdp_w4_q2.log | head -4; tail -2 $OUT/rehearsal_gpt2_fsdp_w4_q2.log
  exit $rc
fi
exit 0
