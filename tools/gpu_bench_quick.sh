# quick bench (no PMC, no CPU baseline) + kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_quick.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_quick -o bench --output-format csv -- python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/prof_quick.log 2>&1
