#!/bin/bash
# rocprofv3 PMC counter passes over the hand-written kernels (kernel-trace only, no sys/runtime traces).
set -u
PROBE=${PROBE:-scripts/pmc_kernels.py}
export PYTHONPATH=.
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python $PROBE > $OUT/probe_plain.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace -d $OUT/pmc_a -o a --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -- python3 $PROBE > $OUT/pmc_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace -d $OUT/pmc_b -o b --output-format csv --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -- python3 $PROBE > $OUT/pmc_b.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace -d $OUT/pmc_c -o c --output-format csv --pmc FETCH_SIZE GRBM_GUI_ACTIVE -- python3 $PROBE > $OUT/pmc_c.log 2>&1 || exit $?
python3 scripts/summarize_pmc.py $OUT > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt | cut -c1-220
