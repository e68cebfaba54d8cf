#!/bin/bash
# Round-3 GPU session 5: fork in-place fix (ResNet tests, breakdown, bench), PMC passes over the flagship
# attention kernels + hand TT GEMM + hipBLASLt NT, world-4 one-GPU rehearsal with 2 queues per rank.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "resnet or conv1x1 or batchnorm" -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/r3_pytest_resnet.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 $OUT/r3_pytest_resnet.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/resnet_kernel_breakdown.py > $OUT/r3_resnet50_kernel_breakdown_fork.jsonl 2> $OUT/r3_resnet50_kernel_breakdown_fork.err
rc=$?; echo "resnet breakdown rc=$rc"; head -n 14 $OUT/r3_resnet50_kernel_breakdown_fork.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload resnet50-ddp > $OUT/r3_bench_resnet.json 2> $OUT/r3_bench_resnet.err
rc=$?; echo "bench resnet rc=$rc"; tail -c 400 $OUT/r3_bench_resnet.json; [ $rc -eq 0 ] || exit $rc
PROBE=scripts/pmc_r3.py bash scripts/gpu_pmc.sh > $OUT/r3_pmc_run.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -n 8 $OUT/r3_pmc_run.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
WORLDS="4" bash scripts/gpu_rehearsal.sh
exit $?
