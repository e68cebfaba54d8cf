#!/bin/bash
# TunableOp GEMM search for the flagship step (hipBLASLt + rocBLAS candidates per GEMM shape), then the
# bench with the tuned table (read-only) vs without.  A heartbeat file keeps the silent tuning pass alive.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( for i in $(seq 1 60); do sleep 30; echo "tick $i" >> $OUT/tune_heartbeat.log; done ) &
HB=$!
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_gfx950.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=15
export PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=0
timeout -k 10 900 python bench.py --micro-batch 32 --steps 1 --warmup 1 > $OUT/tune_pass.log 2>&1; rc=$?
echo "tune rc=$rc"; tail -n 3 $OUT/tune_pass.log
[ $rc -eq 0 ] || { kill $HB; exit $rc; }
ls -la $OUT/tunableop_gfx950*.csv
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 300 python bench.py --micro-batch 32 --steps 6 --warmup 2 2> $OUT/tuned.err; rc=$?
tail -n 1 $OUT/tuned.err
PYTORCH_TUNABLEOP_ENABLED=0 timeout -k 10 300 python bench.py --micro-batch 32 --steps 6 --warmup 2 2> $OUT/untuned.err
tail -n 1 $OUT/untuned.err
kill $HB
exit $rc
