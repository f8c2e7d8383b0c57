# Microbench + parity tests + bench (+ optional rocprof) in one GPU call.
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x tools/gemv_bench ]; then
  timeout -k 10 300 ./tools/gemv_bench 1 > gpurun_out/gemv_bench.log 2>&1; echo "rc=$?" >> gpurun_out/gemv_bench.log
  [ "${M4:-0}" = "1" ] && { timeout -k 10 300 ./tools/gemv_bench 4 > gpurun_out/gemv_bench_m4.log 2>&1; echo "rc=$?" >> gpurun_out/gemv_bench_m4.log; }
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python -u bench.py --cpu-baseline 0 > gpurun_out/prof_bench.log 2>&1
  echo "prof rc=$?" >> gpurun_out/prof_bench.log
fi
if [ "${MATRIX:-0}" = "1" ]; then
  timeout -k 10 600 python -u tools/bench_matrix.py > gpurun_out/bench_matrix.log 2>&1
  echo "matrix rc=$?" >> gpurun_out/bench_matrix.log
fi
