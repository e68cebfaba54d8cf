#!/bin/bash
# ResNet-50 with the in-tree MIOpen db (fresh box: how long is the warmup?), stock ResNet-50 / SwinIR with find
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r12; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
echo "=== ours resnet50 (in-tree MIOpen db)"
t0=$(date +%s)
timeout -k 10 500 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 2> $OUT/r12_a.err || exit $?
echo "wall $(( $(date +%s) - t0 )) s"
du -sh ~/.cache/miopen 2>/dev/null || true
echo "=== stock resnet50 (MIOpen find, same db)"
MIOPEN_USER_DB_PATH=$PWD/tuning/miopen timeout -k 10 500 python scripts/bench_torch_baseline.py --workload resnet50-ddp --steps 20 --warmup 5 2> $OUT/r12_b.err || exit $?
echo "=== stock swinir (MIOpen find)"
t0=$(date +%s)
MIOPEN_USER_DB_PATH=$OUT/miopen_swinir timeout -k 10 700 python scripts/bench_torch_baseline.py --workload swinir-stoke --steps 10 --warmup 3 2> $OUT/r12_c.err || exit $?
echo "wall $(( $(date +%s) - t0 )) s"
