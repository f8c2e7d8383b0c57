#!/bin/bash
# serve.py on one GPU (world 1), bloom-1b1: tokens/s and wall time for prompt lengths 16 / 128 / 512
# (continuous admission feeds a prompt one token per round: ADVICE r2 asks for these figures).
mkdir -p gpurun_out
: > gpurun_out/serve_prompts.log
for P in 16 128 512; do
  timeout -k 10 240 python -m distributed_inference_demo_amd.serve --model bloom-1b1 --num-sample 4 --max-length 32 \
    --core-pool-size 2 --prompt-len $P > gpurun_out/serve_p$P.log 2>&1 || exit 1
  echo "prompt $P: $(tail -1 gpurun_out/serve_p$P.log)" >> gpurun_out/serve_prompts.log
done
