#!/bin/bash
# int8 vs bf16 weights: decode bench lines + a kernel-trace profile of the int8 7b1 run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 240 python bench.py --cpu-baseline 0 --no-pmc --steps 64 --warmup 8 "$@" >> gpurun_out/int8_bench.log 2>&1; }
: > gpurun_out/int8_bench.log
for cfg in "--model bloom-1b1 --batch 1 --prompt 512" "--model bloom-7b1 --batch 1 --prompt 128" \
           "--model bloom-7b1 --batch 4 --prompt 128" "--model bloom-3b --batch 1 --prompt 64"; do
  for w in bf16 int8; do
    echo "== $cfg --weights $w" >> gpurun_out/int8_bench.log
    run $cfg --weights $w || exit 1
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_int8 -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 32 --warmup 4 --model bloom-7b1 \
  --batch 1 --prompt 128 --weights int8 > $GRAFT_REPO_ROOT/gpurun_out/prof_int8.log 2>&1
