# rocprofv3 kernel stats of bench.py under two env settings (A/B): $1 = env assignment for B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profA -o run --output-format csv -- python -u bench.py --cpu-baseline 0 --no-pmc --steps 32 > gpurun_out/profA.log 2>&1 || exit $?
export ${1:-BS_QKV_ATTN=0}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o run --output-format csv -- python -u bench.py --cpu-baseline 0 --no-pmc --steps 32 > gpurun_out/profB.log 2>&1 || exit $?
