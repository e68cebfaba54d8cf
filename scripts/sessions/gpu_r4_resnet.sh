#!/bin/bash
# Round 4: ResNet-50 DDP host overhead -- the bench, then the same run under cProfile (host hotspots).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_resnet${TAG:-}
mkdir -p $OUT
echo "=== resnet bench"; date
timeout -k 10 300 python -u bench.py --workload resnet50-ddp --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
echo "=== cprofile"; date
timeout -k 10 300 python -u -m cProfile -o $OUT/resnet.prof bench.py --workload resnet50-ddp --steps 20 --warmup 3 > $OUT/cprof_bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $OUT/cprof_bench.log; [ $rc -eq 0 ] || exit $rc
python - <<'PY' > $OUT/cprof_top.txt
import pstats
p = pstats.Stats("gpurun_out/r4_resnet%s/resnet.prof" % __import__("os").environ.get("TAG", ""))
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(45)
PY
head -80 $OUT/cprof_top.txt
