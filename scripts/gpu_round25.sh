#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in 3 4 5 6; do
echo "=== PDT_FA_BWD=$v"
PDT_FA_BWD=$v timeout -k 10 200 python scripts/attn_causal_probe.py 2>&1 | grep '^{' || exit 1
done
