#!/bin/bash
# Round 4: GEMM tile-walk group height A/B (PDT_GEMM_GRP) on the NT shapes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_grp
mkdir -p $OUT
for g in 1 2 4 8 16; do
  echo "=== grp $g"
  PDT_GEMM_GRP=$g MODE=bench ROUNDS=3 ONLY=${ONLY:-} timeout -k 10 300 python -u scripts/bench_gemm_asm.py > $OUT/g$g.jsonl 2> $OUT/g$g.err
  rc=$?; echo "rc=$rc"; grep nt_ $OUT/g$g.jsonl | cut -c1-140; [ $rc -eq 0 ] || exit $rc
done
