#!/bin/bash
# Round-4: HIP-graph capture of hook-driven RCCL bucket all-reduces (world > 1 DDP path), then the PMC passes.
set -u
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k graphed -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { tail -n 30 gpurun_out/graph_tests.log; exit 1; }
tail -n 6 gpurun_out/graph_tests.log
bash scripts/sessions/gpu_r4_pmc.sh
