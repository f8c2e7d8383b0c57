#!/bin/bash
# As gpu_r6y.sh at a 1024-token prompt (the decode attention splits, so the merge is deferred or not).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
out=gpurun_out/r6y2.txt
: > $out
for m in bloom-1b1 bloom-3b bloom-7b1; do
  for b in 1 2 4; do
    for t in 4 1; do
      r=$(BS_PARTS_MAX_M=$t timeout -k 10 200 python bench.py --model $m --batch $b --prompt 1024 --steps 64 --warmup 8 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
      echo "$m B=$b prompt 1024 parts_max_m=$t: $r" >> $out
    done
  done
done
