#!/bin/bash
# two query groups per wave in the prefill attention: A/B tool + prefill parity
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 ./tools/attn_prefill_bench > gpurun_out/r5s_attn.txt 2>&1 || exit 1
timeout -k 10 600 $T tests/test_gpu_prefill_split.py tests/test_gpu_7b1_width.py tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_pipeline_7b1.py > gpurun_out/r5s_tests.log 2>&1 || exit 1
