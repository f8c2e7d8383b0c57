#!/bin/bash
# int8 GEMV bytes per lane per step (BS_Q8_CW=16|32) A/B at bloom-7b1 / 3b / 1b1 batch 1, after the int8 tests.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_int8.log 2>&1 || exit 1
BS_Q8_CW=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/gpu_int8.log 2>&1 || exit 1
: > gpurun_out/q8_cw.log
for model in "bloom-7b1 --prompt 128" "bloom-3b --prompt 64" "bloom-1b1 --prompt 512"; do
  for cw in 16 32; do
    echo "== $model BS_Q8_CW=$cw" >> gpurun_out/q8_cw.log
    BS_Q8_CW=$cw timeout -k 10 200 python bench.py --cpu-baseline 0 --no-pmc --steps 64 --warmup 8 --weights int8 \
      --model $model >> gpurun_out/q8_cw.log 2>&1 || exit 1
  done
done
