#!/bin/bash
# batched GEMV table retune: parity (bf16 + int8) and decode rows
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_batched_gemv.py tests/test_gpu_int8.py tests/test_gpu_parity.py -k "batched or small_batch or int8 or ldsw4" > gpurun_out/r5w_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_matrix.py batched --only=bloom-1b1:8,bloom-560m:8,bloom-560m:16,bloom-1b1:32,bloom-560m:32 > gpurun_out/r5w_bm.jsonl 2> gpurun_out/r5w_bm.err || exit 1
