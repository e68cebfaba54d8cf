#!/bin/bash
# Round-3 full GPU check: every pytest -m gpu test, then a kernel-stats profile of the flagship bench config.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT/prof_r3b
timeout -k 10 240 python -u scripts/bench_gemm_diag.py > $OUT/r3_gemm_diag.jsonl 2> $OUT/r3_gemm_diag.err
rc=$?; echo "gemm diag rc=$rc"; cat $OUT/r3_gemm_diag.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $OUT/r3_pytest_gpu_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 $OUT/r3_pytest_gpu_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r3b -o flagship -- python3 bench.py --steps 3 --warmup 2 --secondary 0 > $OUT/r3_prof_flagship_b.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -n 2 $OUT/r3_prof_flagship_b.log; exit $rc
