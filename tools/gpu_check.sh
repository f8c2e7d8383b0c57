mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?" >> gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python -u bench.py --steps 32 --warmup 4 --cpu-steps 4 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/bench.log
fi
