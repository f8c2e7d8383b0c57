#!/bin/bash
# Decode attention split rule at batched sizes (1024-token prompt): blocks targeted (BS_ATT_TARGET 256 / 512) and the
# (row, head) count from which a pair takes one block (BS_ATT_PAIRS_MAX 192 / 384 / 768).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
out=gpurun_out/r6ad.txt
: > $out
for mb in "bloom-1b1 4" "bloom-1b1 8" "bloom-1b1 16" "bloom-7b1 4" "bloom-7b1 8" "bloom-7b1 16"; do
  set -- $mb
  for v in "256 192" "512 192" "512 384" "1024 768"; do
    set -- $mb $v
    r=$(BS_ATT_TARGET=$3 BS_ATT_PAIRS_MAX=$4 timeout -k 10 200 python bench.py --model $1 --batch $2 --prompt 1024 --steps 32 --warmup 4 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
    echo "$1 B=$2 target=$3 pairs_max=$4: $r" >> $out
  done
done
