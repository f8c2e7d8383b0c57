mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemv_bench > gpurun_out/gemv_bench.log 2>&1
echo "rc=$?" >> gpurun_out/gemv_bench.log
