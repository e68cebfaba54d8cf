#!/bin/bash
# Round 6 (q): head-major q/k/v/dO staging for the window-attention backward -- tests, kernel A/B, SwinIR benches.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_q
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "window or swinir or rel" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python3 scripts/bench_window_attn.py | tee $OUT/wa_hm.json
PDT_WIN_HEAD_MAJOR=0 timeout -k 10 120 python3 scripts/bench_window_attn.py | tee $OUT/wa_tm.json
for cfg in "PDT_WIN_HEAD_MAJOR=0" "PDT_WIN_HEAD_MAJOR=1"; do
  for extra in "" "--precision fp32"; do
    env $cfg timeout -k 10 300 python3 bench.py --workload swinir-stoke --loss feat --steps 20 --warmup 5 $extra > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
    echo "$cfg $extra: $(grep '^{' $OUT/b.log | tail -1 | cut -c1-160)" | tee -a $OUT/bench.txt
  done
done
exit 0
