#!/bin/bash
# Prefill changes (GEMM dispatch + split-K, split-KV attention): GPU tests, kernel trace by grid, bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefill_split.py tests/test_gpu_full_size.py tests/test_gpu_7b1_width.py tests/test_gpu_parity.py -v -x --timeout 150 --timeout-method thread > gpurun_out/pf_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pf_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_trace_prefill.sh pf > /dev/null || exit 1
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-pmc --cpu-baseline 0 > gpurun_out/pf_bench.json 2> gpurun_out/pf_bench.err || exit 1
