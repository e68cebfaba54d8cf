#!/bin/bash
# Round 5 (p): GEMM start stagger (PDT_GEMM_STAGGER, 100 MHz ticks per phase group) on the c_fc / c_proj shapes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_p${TAG:-}
mkdir -p $OUT
for st in 0 1200 600 2400 0; do
  echo "=== stagger $st"
  PDT_GEMM_STAGGER=$st MODE=bench ONLY=fc ROUNDS=4 timeout -k 10 180 python3 scripts/bench_gemm_asm.py > $OUT/st$st.log 2>&1 || exit $?
  cat $OUT/st$st.log | grep '^{'
done
exit 0
# (the PDT_GEMM_STAGGER knob this measured was removed after the run)
