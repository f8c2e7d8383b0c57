#!/bin/bash
# After the tile-GEMV rule: the whole GPU suite, then decode at B = 2 / 4 on the three models.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6x_tests.log 2>&1 || exit 1
out=gpurun_out/r6x_bench.txt
: > $out
for m in bloom-1b1 bloom-3b bloom-7b1; do
  for b in 2 4; do
    r=$(timeout -k 10 200 python bench.py --model $m --batch $b --prompt 128 --steps 64 --warmup 8 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
    echo "$m B=$b: $r" >> $out
  done
done
