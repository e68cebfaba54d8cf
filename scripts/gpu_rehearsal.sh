#!/bin/bash
# Multi-rank rehearsal on ONE MI355X (ranks share cuda:0; device collectives on the peer-mapped xGMI kernels,
# bootstrap + object collectives on gloo -- RCCL needs one GPU per rank).  A plumbing check of the N-rank
# engine paths, not a measurement.  Every GPU step has its own time limit; the script stops at the first
# failure.  Logs land in gpurun_out/.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
WORLDS=${WORLDS:-"4"}
# HIP's default hardware queues per rank (4): since round 4 at most ONE wave per rank waits on the mesh (the
# round-3 kernels spun in every workgroup and a late rank's kernels could sit behind its peers' spinners:
# profiles/r3_rehearsal_gpt2_fsdp_w4_q4_vs_q2.log).  The headline guard is relaxed: ranks share one device.
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-4}
export PDT_BENCH_REHEARSAL=1
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 $OUT/$name.log
  return $rc
}
for W in $WORLDS; do
  PDT_BENCH_BACKEND=gloo PDT_XGMI=1 run rehearsal_gpt2_fsdp_w$W 300 \
    python bench.py --gpus $W --micro-batch 2 --steps 3 --warmup 1 --secondary-micro-batch 8 || exit $?
  PDT_BENCH_BACKEND=gloo PDT_XGMI=1 run rehearsal_swinir_stoke_w$W 300 \
    python bench.py --gpus $W --workload swinir-stoke --micro-batch 4 --steps 3 --warmup 1 || exit $?
done
exit 0
