# GPU tests, quick bench (no PMC / CPU baseline) with kernel stats, serve CLI, driver smoke
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_quick.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_quick -o bench --output-format csv -- python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/prof_quick.log 2>&1 || exit $?
timeout -k 10 300 python -u -m distributed_inference_demo_amd.serve --model bloom-560m --num-sample 6 --max-length 32 --core-pool-size 3 > gpurun_out/serve_560m.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
