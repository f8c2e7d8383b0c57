# PMC pass (its own run, kernel counters only): HBM fetch/write bytes per dispatch.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- python -u bench.py --steps 16 --warmup 2 --cpu-baseline 0 --no-profile > gpurun_out/pmc_fetch.log 2>&1
echo "pmc fetch rc=$?" >> gpurun_out/pmc_fetch.log
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc -o write --output-format csv -- python -u bench.py --steps 16 --warmup 2 --cpu-baseline 0 --no-profile > gpurun_out/pmc_write.log 2>&1
echo "pmc write rc=$?" >> gpurun_out/pmc_write.log
