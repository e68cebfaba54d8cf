#!/bin/bash
# full GPU regression: pytest -m gpu, smoke(), default bench
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/full_pytest.log 2>&1 || { tail -40 $OUT/full_pytest.log; exit 1; }
tail -2 $OUT/full_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 || exit 1
timeout -k 10 600 python bench.py 2> $OUT/full_bench.err || exit $?
