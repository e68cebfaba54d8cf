#!/bin/bash
# GEMM role microbench (which flagship GEMM is slow), then the full GPU regression suite + smoke + bench
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 python -u scripts/bench_gemm_roles.py > $OUT/r28_gemm_roles.jsonl 2> $OUT/r28_gemm_roles.err || { tail $OUT/r28_gemm_roles.err; exit 1; }
cat $OUT/r28_gemm_roles.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/r28_pytest.log 2>&1 || { tail -40 $OUT/r28_pytest.log; exit 1; }
tail -2 $OUT/r28_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r28_smoke.log 2>&1 || { tail $OUT/r28_smoke.log; exit 1; }
tail -1 $OUT/r28_smoke.log
timeout -k 10 600 python bench.py 2> $OUT/r28_bench.err || exit $?
