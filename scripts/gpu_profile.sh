#!/bin/bash
# rocprofv3 evidence run: kernel stats of the flagship step + PMC counters of the attention kernels
# and the LayerNorm kernels.  Counter runs use --pmc with kernel-trace only (no sys/runtime traces).
set -u
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 > $OUT/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/pmcA -o attn --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -- python3 scripts/pmc_attention.py > $OUT/pmcA.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/pmcB -o attn --output-format csv --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -- python3 scripts/pmc_attention.py > $OUT/pmcB.log 2>&1 || exit $?
python3 scripts/summarize_prof.py $OUT
