#!/bin/bash
# Head (ln_f + lm_head + pick) at M = 2..4: the rows GEMV's LayerNorm-fused argmax vs the tile path (BS_HEAD_TILES=1).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
out=gpurun_out/r6af.txt
: > $out
for m in bloom-1b1 bloom-3b bloom-7b1; do
  for b in 2 3 4; do
    for t in 0 1; do
      r=$(BS_HEAD_TILES=$t timeout -k 10 200 python bench.py --model $m --batch $b --prompt 128 --steps 64 --warmup 8 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
      echo "$m B=$b head_tiles=$t: $r" >> $out
    done
  done
done
