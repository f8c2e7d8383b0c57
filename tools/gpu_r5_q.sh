#!/bin/bash
# 128 x 96 GEMM tiles in the dispatch: prefill parity + bench prefill
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_prefill_split.py tests/test_gpu_7b1_width.py tests/test_gpu_parity.py tests/test_gpu_full_size.py > gpurun_out/r5q_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --no-configs > gpurun_out/r5q_bench.json 2> gpurun_out/r5q_bench.err || exit 1
