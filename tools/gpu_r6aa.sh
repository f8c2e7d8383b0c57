#!/bin/bash
# LayerNorm fused into the batched GEMV's prologue (gemv_ldsw4 LNS) vs the LayerNorm launch + plain tile GEMV
# (BS_LNS_MAX_M = 16 / 0), single-stage decode, same box.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
out=gpurun_out/r6aa.txt
: > $out
for m in bloom-560m bloom-1b1 bloom-3b; do
  for b in 3 4 8 16; do
    for t in 16 0; do
      r=$(BS_LNS_MAX_M=$t timeout -k 10 200 python bench.py --model $m --batch $b --prompt 128 --steps 64 --warmup 8 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
      echo "$m B=$b lns_max_m=$t: $r" >> $out
    done
  done
done
