#!/bin/bash
# ResNet-50: MIOpen solver selection modes (heuristic vs find vs exhaustive search into an in-repo db)
set -u
OUT=gpurun_out
mkdir -p $OUT/miopen_db
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_miopen; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
run() { echo "=== $1"; shift; env "$@" timeout -k 10 600 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 2>> $OUT/miopen.err; }
run default PDT_CONV_BENCHMARK=0 || exit $?
run find_benchmark PDT_CONV_BENCHMARK=1 MIOPEN_USER_DB_PATH=$OUT/miopen_db_find || exit $?
run search PDT_CONV_BENCHMARK=1 MIOPEN_FIND_ENFORCE=3 MIOPEN_USER_DB_PATH=$OUT/miopen_db || exit $?
run after_search PDT_CONV_BENCHMARK=1 MIOPEN_USER_DB_PATH=$OUT/miopen_db || exit $?
run after_search_nobench PDT_CONV_BENCHMARK=0 MIOPEN_USER_DB_PATH=$OUT/miopen_db || exit $?
ls -la $OUT/miopen_db
