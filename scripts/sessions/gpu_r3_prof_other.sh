#!/bin/bash
# Kernel-stats + idle-gap profiles of the non-flagship bench workloads (ResNet-50 DDP, GPT-2 124M DDP):
# where does the GPU sit idle between dispatches?  Stops at the first failing GPU step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for w in ${WORKLOADS:-resnet50-ddp gpt2-ddp}; do
  mkdir -p $OUT/po_$w
  echo "=== $w"; date
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/po_$w -o prof -- python3 bench.py --workload $w --steps 5 --warmup 3 > $OUT/po_$w.log 2>&1
  rc=$?
  echo "=== $w rc=$rc"; tail -n 2 $OUT/po_$w.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
  db=$(find $OUT/po_$w -name "*.db" | head -n 1)
  python scripts/prof_db_stats.py "$db" --step-kernel adamw_mt_kernel --skip 3 --gaps 25 -o $OUT/po_${w}_stats.csv > $OUT/po_${w}_table.txt 2>&1 || true
  rm -f "$db"
  grep "#" $OUT/po_${w}_table.txt | head -n 14 | cut -c1-220
  head -n 16 $OUT/po_${w}_stats.csv | cut -c1-160
done
exit 0
