#!/bin/bash
# Full GPU regression + flagship bench/profile + stock baseline at the new default batch + train CLI.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $OUT/r6_pytest.log 2>&1; rc=$?
grep -E "FAIL|Error" $OUT/r6_pytest.log | head -20; tail -n 2 $OUT/r6_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit $?
echo "=== bench (default)"
timeout -k 10 300 python bench.py 2> $OUT/r6_bench.err || exit $?
tail -n 1 $OUT/r6_bench.err
echo "=== stock gpt2 mb32"
timeout -k 10 300 python scripts/bench_torch_baseline.py --workload gpt2-fsdp --micro-batch 32 --steps 6 --warmup 2 2> $OUT/r6_stock.err || exit $?
tail -n 1 $OUT/r6_stock.err
echo "=== train CLI swinir"
timeout -k 10 300 python -m pytorch_distributedtraining_amd.train --config configs/swinir_stoke.yaml --steps 4 2>&1 | grep -v amdgpu.ids | tail -n 3 || exit $?
echo "=== rocprof flagship"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_flag -o flag --output-format csv -- python3 bench.py --steps 3 --warmup 1 > $OUT/prof_flag.log 2>&1 || exit $?
python3 scripts/trace_kernels.py $(find $OUT/prof_flag -name "*kernel_trace.csv" | head -1) --top 25
