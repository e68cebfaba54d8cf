#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_wgrad_variants.py > $OUT/r31_wgrad.jsonl 2> $OUT/r31_wgrad.err || { tail $OUT/r31_wgrad.err; exit 1; }
cat $OUT/r31_wgrad.jsonl
