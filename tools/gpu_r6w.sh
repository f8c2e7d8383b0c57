#!/bin/bash
# Tile GEMV from M = 2 / 3 / 4 (BS_TILES_MIN_M) against the default (5): GEMV probe both ways, then decode at
# B = 2 / 3 / 4 on bloom-1b1, 3b and 7b1 (single stage, graph decode) both ways, same box.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
out=gpurun_out/r6w.txt
: > $out
timeout -k 10 150 ./tools/rows_m_probe >> $out 2>&1 || exit 1
BS_TILES_MIN_M=2 timeout -k 10 150 ./tools/rows_m_probe >> $out 2>&1 || exit 1
for m in bloom-1b1 bloom-3b bloom-7b1; do
  for b in 2 3 4; do
    for t in 5 2 3; do
      r=$(BS_TILES_MIN_M=$t timeout -k 10 200 python bench.py --model $m --batch $b --prompt 128 --steps 64 --warmup 8 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
      echo "$m B=$b tiles_min_m=$t: $r" >> $out
    done
  done
done
