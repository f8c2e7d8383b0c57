#!/bin/bash
# Prefill GEMM iteration: K-step probes, the dispatch back to back, block stamps, then the GPU tests that reach
# the GEMMs (prefill parity at every family width, pipeline splits).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/kstep_probe2 > gpurun_out/gi_kstep2.txt 2>&1 || exit 1
timeout -k 10 200 ./tools/gemm_splitk_bench > gpurun_out/gi_b2b.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/gemm3_stamps > gpurun_out/gi_stamps.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_7b1_width.py tests/test_gpu_prefill_split.py tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gi_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gi_pytest.log; exit $rc
