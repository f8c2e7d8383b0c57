# rocprofv3 kernel stats of one bench configuration: MODEL BATCH PROMPT [TAG]
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${4:-cfg}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 -u bench.py --model $1 --batch $2 --prompt $3 --steps 16 --warmup 2 --cpu-baseline 0 --no-pmc > gpurun_out/prof_$TAG.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof_$TAG.log
