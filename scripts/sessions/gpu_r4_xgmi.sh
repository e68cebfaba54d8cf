#!/bin/bash
# Round 4: xGMI mesh with one waiting workgroup per rank (+ any-size / fp64 latency class) -- GPU tests.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_xgmi${TAG:-}
mkdir -p $OUT
echo "=== xgmi tests"; date
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_xgmi_gpu.py \
  tests/test_xgmi_engines_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "xgmi rc=$rc"; tail -25 $OUT/pytest.log
exit $rc
