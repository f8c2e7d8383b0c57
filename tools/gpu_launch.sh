# Launch-engine iteration: GPU parity suite, bench, and a rocprofv3 kernel trace of the bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 64 --warmup 4 --cpu-baseline 0 --no-pmc > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python -u bench.py --steps 32 --warmup 4 --cpu-baseline 0 --no-pmc --no-profile > gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof_bench.log
