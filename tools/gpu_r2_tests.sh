# round 2: GPU test suite (new + full-size parity first), then the rest, quick bench + kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_rows_sampling.py -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
echo "new rc=$?" >> gpurun_out/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread --deselect tests/test_gpu_full_size.py --deselect tests/test_gpu_rows_sampling.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_quick.log 2>&1 || exit $?
