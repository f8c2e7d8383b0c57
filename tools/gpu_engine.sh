# Persistent decode engine: its parity tests first (fail fast), a phase trace, then the full GPU
# suite and the bench on both engines.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1
rc=$?
echo "engine pytest rc=$rc" >> gpurun_out/pytest_engine.log
[ $rc -eq 0 ] || exit $rc
BS_ENGINE_TRACE=1 timeout -k 10 120 python -u tools/engine_trace.py bloom-1b1 1 512 > gpurun_out/engine_trace.log 2>&1
echo "trace rc=$?" >> gpurun_out/engine_trace.log
timeout -k 10 300 python -u bench.py --steps 64 --warmup 4 --cpu-baseline 0 --no-pmc > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 64 --warmup 4 --cpu-baseline 0 --no-pmc --engine launches > gpurun_out/bench_launches.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_launches.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
