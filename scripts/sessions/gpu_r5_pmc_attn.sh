#!/bin/bash
# Round 5: PMC passes over the flagship-shape attention (B96 S1024 H16 D128 causal, packed qkv + bias gradient).
set -u
export TMPDIR=/tmp ROUNDS=1
OUT=gpurun_out/r5_pmc_attn${TAG:-} PROBE=scripts/bench_attn_flagship.py bash scripts/gpu_pmc.sh
