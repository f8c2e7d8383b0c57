# Batched probe + parity tests + config matrix in one GPU call.
mkdir -p gpurun_out
export TMPDIR=/tmp
PROBE_BATCH=1 timeout -k 10 200 ./tools/gemv_probe > gpurun_out/gemv_probe_batch.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/bench_matrix.py > gpurun_out/bench_matrix.log 2>&1
echo "matrix rc=$?" >> gpurun_out/bench_matrix.log
