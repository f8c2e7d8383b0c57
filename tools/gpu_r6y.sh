#!/bin/bash
# Deferred attention merge (dense rows GEMV merges the split partials) vs the attention's own ticket merge + the tile
# dense GEMV, at B = 2..4 (BS_PARTS_MAX_M = 4 / 2 / 1), same box.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
out=gpurun_out/r6y.txt
: > $out
for m in bloom-1b1 bloom-3b bloom-7b1; do
  for b in 2 3 4; do
    for t in 4 2 1; do
      r=$(BS_PARTS_MAX_M=$t timeout -k 10 200 python bench.py --model $m --batch $b --prompt 128 --steps 64 --warmup 8 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
      echo "$m B=$b parts_max_m=$t: $r" >> $out
    done
  done
done
