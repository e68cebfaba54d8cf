#!/bin/bash
# Generic GPU step runner: each argument is "name|timeout_s|command"; steps run in order, each under its own
# time limit, output to gpurun_out/<name>.log; stops at the first step that fails with a GPU-fatal status
# (abort / segfault / timeout) and, unless KEEP_GOING=1, at any failure.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 8 "$OUT/$name.log"
  case $rc in
    0) ;;
    124|134|137|139) echo "GPU-fatal status $rc: stopping"; exit $rc ;;
    *) [ "${KEEP_GOING:-0}" = "1" ] || exit $rc ;;
  esac
done
