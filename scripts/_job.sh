set -o pipefail
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_bisect.py || exit $?
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x -k "flash or swinir" > gpurun_out/k_test.log 2>&1; rc=$?
tail -3 gpurun_out/k_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_kernels.py --only attnvar,attn > gpurun_out/fa_bench.log 2>&1 || exit $?
cat gpurun_out/fa_bench.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 2> gpurun_out/bench.err || exit $?
