#!/bin/bash
# batched GEMV: no duplicate B-row loads, LN prologue with DPP-broadcast gamma/beta: sweep, parity, decode rows
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 ./tools/tiles_bench > gpurun_out/r5l_tiles.txt 2>&1 || exit 1
timeout -k 10 420 $T tests/test_gpu_batched_gemv.py > gpurun_out/r5l_batched.log 2>&1 || exit 1
timeout -k 10 420 $T tests/test_gpu_parity.py -k "batched or small_batch" > gpurun_out/r5l_parity.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_matrix.py batched --only=bloom-1b1:8,bloom-560m:8,bloom-560m:16,bloom-3b:8,bloom-1b1:32,bloom-560m:32 > gpurun_out/r5l_bm.jsonl 2> gpurun_out/r5l_bm.err || exit 1
