#!/bin/bash
# Round 6 (e): micro-batch headroom on 288 GB -- flagship GPT-2 1.3B FSDP at 96 / 112 / 128 sequences per GPU and
# Llama-3 8B config 5 (selective recompute on all layers) at 16 / 24 / 32, plus the fake-world-8 rehearsal
# with real values in the collective outputs.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_e
mkdir -p $OUT
run() {  # name, timeout, args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', d.get('value'), d.get('ms_per_step'), d.get('peak_mem_gb'))"
}
run gpt2_mb96 300 --steps 6 --warmup 2 --secondary 0 --overlap-probe 0 || exit 1
run gpt2_mb112 300 --steps 6 --warmup 2 --secondary 0 --overlap-probe 0 --micro-batch 112 || true
run gpt2_mb128 300 --steps 6 --warmup 2 --secondary 0 --overlap-probe 0 --micro-batch 128 || true
run fake8_gpt2 300 --rehearse-world 8 --steps 6 --warmup 2 || exit 1
run llama_mb16 400 --workload llama3-fsdp --steps 4 --warmup 2 --overlap-probe 0 || exit 1
run llama_mb24 400 --workload llama3-fsdp --steps 4 --warmup 2 --overlap-probe 0 --micro-batch 24 || true
run llama_mb32 400 --workload llama3-fsdp --steps 4 --warmup 2 --overlap-probe 0 --micro-batch 32 || true
OUT=gpurun_out/r6_e_pmc PROBE=scripts/pmc_window.py bash scripts/gpu_pmc.sh || exit $?
exit 0
