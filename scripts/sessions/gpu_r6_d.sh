#!/bin/bash
# Round 6 (d): world-8 readiness on one GPU through torch's fake process group -- the GPU test module, then the
# bench.py rehearsal lines (per-rank compute ms/step, collectives and peak memory at fake world 8) of the
# flagship, ResNet-50 DDP and SwinIR Stoke, against the flagship at N = 1.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_fake_world8_gpu.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "PASSED|FAILED|fake world|passed|failed" $OUT/pytest.log | tail -12
run() {  # name, timeout, args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  cut -c1-420 $OUT/$name.json
}
run n1_gpt2 300 --steps 6 --warmup 2 --secondary 0 --overlap-probe 0 || exit 1
run fake8_gpt2_r7 300 --rehearse-world 8 --steps 6 --warmup 2 || exit 1
run fake8_gpt2_r0 300 --rehearse-world 8 --rehearse-rank 0 --steps 6 --warmup 2 || exit 1
run fake8_resnet 300 --rehearse-world 8 --workload resnet50-ddp --steps 6 --warmup 2 || exit 1
run fake8_swinir 300 --rehearse-world 8 --workload swinir-stoke --steps 6 --warmup 2 || exit 1
exit 0
