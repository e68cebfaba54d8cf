#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/attn_causal_probe.py 2>&1 | grep '^{' 
