#!/bin/bash
# Round 6: the four-m-tile fc2 rule (K >= 4N, 33..64 tokens) at the other widths: serve.py --max-length 0, one
# 64- / 48-token sample a pass, BS_TILES_MAX_M=32 (fc2 on the prefill GEMM) vs the default.
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
for model in bloom-560m bloom-3b bloom-7b1; do
  for plen in 64 40; do
    for mm in 32 64; do
      BS_TILES_MAX_M=$mm timeout -k 10 200 python -u -m distributed_inference_demo_amd.serve --model $model --max-length 0 \
        --n-labels 2 --num-sample 128 --prompt-len $plen --core-pool-size 1 > gpurun_out/r6ad_${model}_${plen}_m$mm.log 2>&1 || exit 1
      echo "$model prompt $plen BS_TILES_MAX_M=$mm $(tail -1 gpurun_out/r6ad_${model}_${plen}_m$mm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["samples_per_s"],1), "samples/s")')"
    done
  done
done
