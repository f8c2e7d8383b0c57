#!/bin/bash
# int8 GEMV rows-per-wave sweep (BS_Q8_R) at bloom-7b1 / bloom-1b1 batch 1.
mkdir -p gpurun_out
: > gpurun_out/q8_sweep.log
for model in "bloom-7b1 --prompt 128" "bloom-1b1 --prompt 512"; do
  for r in 0 1 2 4; do
    echo "== $model BS_Q8_R=$r" >> gpurun_out/q8_sweep.log
    BS_Q8_R=$r timeout -k 10 200 python bench.py --cpu-baseline 0 --no-pmc --steps 64 --warmup 8 --weights int8 \
      --model $model >> gpurun_out/q8_sweep.log 2>&1 || exit 1
  done
done
