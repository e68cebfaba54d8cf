#!/bin/bash
# Round 4: ResNet-50 DDP host overhead -- un-profiled ms/step, host ms/step, torch-profiler CPU self time.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r4_resnet${TAG:-}
mkdir -p $OUT
echo "=== resnet host profile"; date
timeout -k 10 400 python -u scripts/resnet_host_prof.py > $OUT/host_prof.txt 2> $OUT/host_prof.err
rc=$?; echo "rc=$rc"; head -70 $OUT/host_prof.txt; tail -3 $OUT/host_prof.err
exit $rc
