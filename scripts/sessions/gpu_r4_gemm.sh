#!/bin/bash
# Round 4: hand-scheduled GEMM main loop -- correctness vs the compiler-scheduled kernel / fp32, then timing.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_gemm${TAG:-}
mkdir -p $OUT
echo "=== check"; date
MODE=check timeout -k 10 300 python -u scripts/bench_gemm_asm.py > $OUT/check.jsonl 2> $OUT/check.err
rc=$?; echo "check rc=$rc"; cat $OUT/check.jsonl; tail -5 $OUT/check.err
[ $rc -eq 0 ] || exit $rc
echo "=== check, 3-stage program forced"; date
PDT_GEMM_P3=1 MODE=check timeout -k 10 300 python -u scripts/bench_gemm_asm.py > $OUT/check_p3.jsonl 2> $OUT/check_p3.err
rc=$?; echo "check_p3 rc=$rc"; grep -E "false|tails" $OUT/check_p3.jsonl; tail -5 $OUT/check_p3.err
[ $rc -eq 0 ] || exit $rc
echo "=== bench, 3-stage program off (A/B)"; date
PDT_GEMM_P3=0 MODE=bench ROUNDS=${ROUNDS:-5} timeout -k 10 500 python -u scripts/bench_gemm_asm.py > $OUT/bench_p3off.jsonl 2> $OUT/bench_p3off.err
rc=$?; echo "bench_p3off rc=$rc"; cat $OUT/bench_p3off.jsonl
[ $rc -eq 0 ] || exit $rc
echo "=== bench"; date
MODE=bench ROUNDS=${ROUNDS:-5} timeout -k 10 500 python -u scripts/bench_gemm_asm.py > $OUT/bench.jsonl 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.jsonl; tail -5 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
echo "=== stamps"; date
timeout -k 10 200 python -u scripts/gemm_stamps.py > $OUT/stamps.jsonl 2> $OUT/stamps.err
rc=$?; echo "stamps rc=$rc"; cat $OUT/stamps.jsonl; tail -3 $OUT/stamps.err
exit $rc
