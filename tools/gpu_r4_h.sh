#!/bin/bash
# Round 4: prefill attention with 32-query blocks (QW = 2) against 64-query blocks: the kernel bench, then the
# prefill parity tests (the library still dispatches QW = 4).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/attn_prefill_bench > gpurun_out/rh_attn.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_prefill_split.py tests/test_gpu_parity.py tests/test_gpu_7b1_width.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rh_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rh_pytest.log; exit $rc
