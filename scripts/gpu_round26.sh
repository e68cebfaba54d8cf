#!/bin/bash
# flagship kernel profile after the causal heavy-first ordering + attention PMC pass
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
( while true; do date > $OUT/heartbeat_r26; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_flag2 -o f --output-format csv -- python3 bench.py --steps 3 --warmup 1 > $OUT/prof_flag2.log 2>&1 || exit $?
grep '"metric"' $OUT/prof_flag2.log | cut -c1-200
timeout -s KILL 120 rocprofv3 --kernel-trace -d $OUT/pmc_a -o a --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -- python3 scripts/kernel_probe.py > $OUT/pmc_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace -d $OUT/pmc_b -o b --output-format csv --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -- python3 scripts/kernel_probe.py > $OUT/pmc_b.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace -d $OUT/pmc_c -o c --output-format csv --pmc FETCH_SIZE GRBM_GUI_ACTIVE -- python3 scripts/kernel_probe.py > $OUT/pmc_c.log 2>&1 || exit $?
python3 scripts/summarize_pmc.py $OUT > $OUT/pmc_summary.txt
