#!/bin/bash
# Round-3 GPU session 4: BN backward mask-from-x + wide combine (tests + ResNet-50 breakdown + bench with the
# secondary), attention tests with the size-based grouping, world-4 one-GPU rehearsal with the queue cap logged.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "batchnorm or flash_attn or resnet or conv1x1" -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/r3_pytest_bn_attn.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 $OUT/r3_pytest_bn_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/trace_resnet_kernels.py > $OUT/r3_resnet50_kernel_breakdown_bn2.jsonl 2> $OUT/r3_resnet50_kernel_breakdown_bn2.err
rc=$?; echo "resnet breakdown rc=$rc"; head -n 14 $OUT/r3_resnet50_kernel_breakdown_bn2.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/r3_bench_n1_bn.json 2> $OUT/r3_bench_n1_bn.err
rc=$?; echo "bench rc=$rc"; tail -c 700 $OUT/r3_bench_n1_bn.json; [ $rc -eq 0 ] || exit $rc
PDT_XGMI_TIMEOUT_S=30 WORLDS="4" bash scripts/gpu_rehearsal.sh
exit $?
