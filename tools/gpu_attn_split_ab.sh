#!/bin/bash
# A/B: decode attention splits (64-position chunks per split: 4 = round 3, 2, 1) on the default bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/asab.txt
for C in 4 2 1 4 2 1; do
  BS_AB_ATTN_CPS=$C timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-pipeline-n1 --cpu-baseline 0 --no-pmc > gpurun_out/asab_$C.json 2>>gpurun_out/asab.err || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/asab_$C.json').read()); print('cps $C', r['value'], r['ms_per_step'])" >> gpurun_out/asab.txt
done
