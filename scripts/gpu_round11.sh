#!/bin/bash
# wave-per-window attention kernels: numerics, SwinIR end-to-end; ResNet-50 / SwinIR stock with MIOpen find
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "window or swinir" > $OUT/r11_pytest.log 2>&1 || { tail -60 $OUT/r11_pytest.log; exit 1; }
tail -3 $OUT/r11_pytest.log
echo "=== ours swinir"
timeout -k 10 400 python bench.py --workload swinir-stoke --steps 20 --warmup 5 2> $OUT/r11_a.err || exit $?
echo "=== ours resnet50"
timeout -k 10 400 python bench.py --workload resnet50-ddp --steps 20 --warmup 5 2> $OUT/r11_b.err || exit $?
echo "=== stock resnet50 (MIOpen find)"
timeout -k 10 400 python scripts/bench_torch_baseline.py --workload resnet50-ddp --steps 20 --warmup 5 2> $OUT/r11_c.err || exit $?
echo "=== stock swinir (MIOpen find)"
timeout -k 10 600 python scripts/bench_torch_baseline.py --workload swinir-stoke --steps 10 --warmup 3 2> $OUT/r11_d.err || exit $?
