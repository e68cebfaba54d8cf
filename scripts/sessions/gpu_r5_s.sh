#!/bin/bash
# Round 5 (s): dQ block order at the flagship attention shape -- default (forward grouped, dQ heavy-first) vs
# PDT_FA_ORDER=5 (dQ grouped per XCD too), and the opt-in persistent dQ, per-kernel times.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_s${TAG:-}
mkdir -p $OUT
for cfg in def ord5 dqp def ord5; do
  echo "=== $cfg"
  unset PDT_FA_ORDER PDT_FA_DQP
  case $cfg in
    ord5) export PDT_FA_ORDER=5 ;;
    dqp) export PDT_FA_DQP=1 ;;
  esac
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$cfg -o a --output-format csv -- python3 scripts/bench_attn_flagship.py > $OUT/$cfg.log 2>&1 || exit $?
  grep '^{' $OUT/$cfg.log
  f=$(find $OUT/$cfg -name "*kernel_stats.csv" | head -1); grep -o '"[^"]*fa_[^"]*",[0-9]*,[0-9]*,[0-9.]*' "$f" | cut -c1-50,120-
done
exit 0
