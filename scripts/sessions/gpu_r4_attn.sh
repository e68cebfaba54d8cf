#!/bin/bash
# Round 4: flash attention -- flagship-shape timing + per-kernel stats, then the attention GPU tests.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_attn${TAG:-}
mkdir -p $OUT
echo "=== attn bench"; date
timeout -k 10 200 python -u scripts/bench_attn_flagship.py > $OUT/bench.jsonl 2> $OUT/bench.err
rc=$?; echo "rc=$rc"; cat $OUT/bench.jsonl; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
echo "=== attn bench, every tile masked (A/B)"; date
PDT_FA_MASK_ALL=1 timeout -k 10 200 python -u scripts/bench_attn_flagship.py > $OUT/bench_maskall.jsonl 2>> $OUT/bench.err
rc=$?; echo "rc=$rc"; cat $OUT/bench_maskall.jsonl; [ $rc -eq 0 ] || exit $rc
echo "=== attn kernel stats"; date
ROUNDS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o attn --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/prof.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
head -8 $(find $OUT/prof -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
echo "=== attn tests"; date
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attn" > $OUT/pytest.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 $OUT/pytest.log
exit $rc
