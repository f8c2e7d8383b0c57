#!/bin/bash
# serve.py on one GPU (world 1), bloom-1b1: tokens/s and wall time for prompt lengths 16 / 128 / 512, with the
# admission prefill pass (default) and with the prompt fed one token a round (--prefill 0, round 3's path).
mkdir -p gpurun_out
: > gpurun_out/serve_prompts.log
for PF in 1 0; do
for P in 16 128 512; do
  timeout -k 10 240 python -m distributed_inference_demo_amd.serve --model bloom-1b1 --num-sample 4 --max-length 32 \
    --core-pool-size 2 --prompt-len $P --prefill $PF > gpurun_out/serve_p${P}_pf$PF.log 2>&1 || exit 1
  echo "prefill $PF prompt $P: $(tail -1 gpurun_out/serve_p${P}_pf$PF.log)" >> gpurun_out/serve_prompts.log
done
done
