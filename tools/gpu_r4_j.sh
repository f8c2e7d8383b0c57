#!/bin/bash
# Round 4: whole-tile 2-stage grids from 384 tiles: GEMM lines, then the prefill / pipeline tests.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/gemm_splitk_bench > gpurun_out/rj_b2b.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_7b1_width.py tests/test_gpu_prefill_split.py tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_pipeline.py tests/test_gpu_pipeline_7b1.py tests/test_gpu_batched_gemv.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rj_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rj_pytest.log; exit $rc
