# rocprofv3 kernel stats of one bench.py run; args passed to bench.py
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python -u bench.py --cpu-baseline 0 --no-pmc --steps 32 "$@" > gpurun_out/prof1.log 2>&1
