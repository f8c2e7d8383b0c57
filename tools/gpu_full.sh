# Round-end evidence: GPU tests, default bench (PMC traffic + CPU baseline), rocprof kernel stats
# of the same command, bench matrix over the BLOOM configs.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o bench --output-format csv -- python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/prof_full.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_matrix.py > gpurun_out/bench_matrix.log 2>&1
echo "matrix rc=$?" >> gpurun_out/bench_matrix.log
