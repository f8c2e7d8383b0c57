# GPU test suite (the driver's round-end tier), logged under gpurun_out/
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; exit $rc
