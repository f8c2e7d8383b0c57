#!/bin/bash
# int8 GEMV: plain activations staged in LDS per block (BS_Q8_XL=1) vs read per wave from L2, A/B.
mkdir -p gpurun_out
BS_Q8_XL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_int8_xl.log 2>&1 || exit 1
: > gpurun_out/q8_xl.log
for model in "bloom-7b1 --prompt 128" "bloom-3b --prompt 64"; do
  for xl in 0 1; do
    echo "== $model BS_Q8_XL=$xl" >> gpurun_out/q8_xl.log
    BS_Q8_XL=$xl timeout -k 10 200 python bench.py --cpu-baseline 0 --no-pmc --steps 64 --warmup 8 --weights int8 \
      --model $model >> gpurun_out/q8_xl.log 2>&1 || exit 1
  done
done
