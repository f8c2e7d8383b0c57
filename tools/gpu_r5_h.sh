#!/bin/bash
# fused attention + dense: parity (bitwise vs separate launches, checker), decode parity suite, headline A/B, host enqueue
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 420 $T tests/test_gpu_attn_dense.py > gpurun_out/r5h_attn_dense.log 2>&1 || exit 1
timeout -k 10 420 $T tests/test_gpu_parity.py -k "decode or split or graph" > gpurun_out/r5h_parity.log 2>&1 || exit 1
for i in 1 2; do
  for f in 0 1; do
    BS_ATTN_DENSE=$f timeout -k 10 240 python3 bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --no-configs > gpurun_out/r5h_b1b1_f${f}_$i.json 2> gpurun_out/r5h_b1b1_f${f}_$i.err || exit 1
  done
done
for f in 0 1; do
  BS_ATTN_DENSE=$f timeout -k 10 240 python3 bench.py --model bloom-560m --cpu-baseline 0 --no-pmc --no-pipeline-n1 --no-configs > gpurun_out/r5h_b560_f${f}.json 2> gpurun_out/r5h_b560_f${f}.err || exit 1
done
N_MB=16 timeout -k 10 200 python3 tools/host_enqueue.py > gpurun_out/r5h_host16.json 2> gpurun_out/r5h_host16.err || exit 1
N_MB=8 timeout -k 10 200 python3 tools/host_enqueue.py > gpurun_out/r5h_host8.json 2> gpurun_out/r5h_host8.err || exit 1
