#!/bin/bash
# After the LN-prologue rule: batched-GEMV tests, then decode at B = 8 / 16 on bloom-1b1 and 3b.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batched_gemv.py tests/test_gpu_parity.py > gpurun_out/r6ab_tests.log 2>&1 || exit 1
out=gpurun_out/r6ab.txt
: > $out
for m in bloom-1b1 bloom-3b; do
  for b in 8 16; do
    r=$(timeout -k 10 200 python bench.py --model $m --batch $b --prompt 128 --steps 64 --warmup 8 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4))") || exit 1
    echo "$m B=$b: $r" >> $out
  done
done
