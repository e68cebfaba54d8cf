#!/bin/bash
# Round-4 PMC passes: shipped attention kernels, the asm GEMM (TT and NT runs separately) and hipBLASLt.
set -u
export PYTHONPATH=.
mkdir -p gpurun_out/pmc4
OUT=gpurun_out/pmc4/all PROBE=scripts/pmc_r4.py MODE=all bash scripts/gpu_pmc.sh || exit $?
OUT=gpurun_out/pmc4/tt PROBE=scripts/pmc_r4.py MODE=tt bash scripts/gpu_pmc.sh || exit $?
OUT=gpurun_out/pmc4/nt PROBE=scripts/pmc_r4.py MODE=nt bash scripts/gpu_pmc.sh || exit $?
