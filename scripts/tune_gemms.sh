#!/bin/bash
# GEMM algorithm selection for the flagship step with PyTorch-ROCm TunableOp (hipBLASLt + rocBLAS
# solution search per GEMM shape).  Pass 1 tunes and writes the table; pass 2 re-runs the bench
# reading it (tuning off) so the two ms/step numbers can be compared.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_gfx950.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-40}
export PYTORCH_TUNABLEOP_VERBOSE=0
echo "== baseline (TunableOp off)"
PYTORCH_TUNABLEOP_ENABLED=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} 2>$OUT/tune_base.err || exit $?
echo "== tuning pass"
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 900 python bench.py --steps 2 --warmup 1 ${BENCH_ARGS:-} > $OUT/tune_pass.log 2>&1 || exit $?
tail -2 $OUT/tune_pass.log
wc -l $PYTORCH_TUNABLEOP_FILENAME
echo "== tuned (read-only)"
PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} 2>$OUT/tune_after.err || exit $?
