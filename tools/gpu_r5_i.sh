#!/bin/bash
# LN prologue in the batched (4 < M <= 16) GEMV: parity + A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 420 $T tests/test_gpu_batched_gemv.py > gpurun_out/r5i_batched.log 2>&1 || exit 1
timeout -k 10 420 $T tests/test_gpu_parity.py -k "batched or small_batch" > gpurun_out/r5i_parity.log 2>&1 || exit 1
O="--only=bloom-1b1:8,bloom-560m:8,bloom-560m:16,bloom-3b:8,bloom-1b1:32,bloom-560m:32"
for i in 1 2; do
  for f in 1 0; do
    BS_LN_UNFUSED=$f timeout -k 10 300 python3 tools/bench_matrix.py batched $O > gpurun_out/r5i_bm_u${f}_$i.jsonl 2> gpurun_out/r5i_bm_u${f}_$i.err || exit 1
  done
done
