#!/bin/bash
# Round 4: two-blocks-per-CU whole-tile GEMM dispatch -- the long-prompt GEMM shapes, then the tests that reach it.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/gemm_splitk_bench > gpurun_out/rf_b2b.txt 2>&1 || exit 1
export BS_PARITY_LOG=$PWD/gpurun_out/rf_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 700 python -u -m pytest tests/test_gpu_7b1_width.py tests/test_gpu_prefill_split.py tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_pipeline.py tests/test_gpu_pipeline_7b1.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rf_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rf_pytest.log; exit $rc
