# prefill changes: GPU tests, bench, narrow-tile A/B, kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_new.log 2>&1 || exit $?
BS_GEMM_NO_NARROW=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_nonarrow.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python -u bench.py --cpu-baseline 0 --no-pmc --steps 32 > gpurun_out/prof1.log 2>&1
