#!/bin/bash
# Round 5 (g): attention per-tile efficiency vs work per workgroup -- the flagship shape against longer
# sequences at the same token count (more key / query tiles per workgroup amortise the prologue / epilogue).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r5_g${TAG:-}
mkdir -p $OUT
run() {  # name, seconds, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep '^{' "$OUT/$name.log" | cut -c1-200
  return $rc
}
run s1k 200 env B=96 S=1024 python scripts/bench_attn_flagship.py || exit $?
run s2k 200 env B=48 S=2048 python scripts/bench_attn_flagship.py || exit $?
run s4k 200 env B=24 S=4096 python scripts/bench_attn_flagship.py || exit $?
run s8k 200 env B=12 S=8192 python scripts/bench_attn_flagship.py || exit $?
exit 0
