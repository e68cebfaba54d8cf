#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_gemm_layouts.py small > $OUT/gemm_small.jsonl 2>&1 || exit $?
grep '^{' $OUT/gemm_small.jsonl
