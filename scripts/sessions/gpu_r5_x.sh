#!/bin/bash
# Round 5 (x): final full check -- pytest -m gpu, smoke, default bench, steady-state flagship kernel table, then
# PMC passes over attention + the GEMM epilogue kernels (scripts/pmc_r4.py).
set -u
export TMPDIR=/tmp
TAG=x bash scripts/sessions/gpu_r5_full.sh || exit $?
OUT=gpurun_out/r5_x_pmc PROBE=scripts/pmc_r4.py bash scripts/gpu_pmc.sh || exit $?
OUT=gpurun_out/r5_x_pmc_dgelu PROBE=scripts/pmc_r4.py MODE=dgelu bash scripts/gpu_pmc.sh || exit $?
exit 0
