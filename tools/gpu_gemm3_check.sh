#!/bin/bash
# gemm_mfma3 in the dispatch: GEMM sweep, the GPU tests that reach it (7b1/3b widths, prefill parity), bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 ./tools/gemm_splitk_bench > gpurun_out/g3_sweep.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_7b1_width.py tests/test_gpu_prefill_split.py tests/test_gpu_parity.py tests/test_gpu_int8.py tests/test_gpu_full_size.py tests/test_gpu_pipeline.py -v -x --timeout 200 --timeout-method thread > gpurun_out/g3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/g3_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-pmc --cpu-baseline 0 > gpurun_out/g3_bench.json 2> gpurun_out/g3_bench.err || exit 1
