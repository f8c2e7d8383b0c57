#!/bin/bash
# Overlapped-attention check: the parity suites that run batch-1 decode, then the headline bench with the overlap on
# and off (same box).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_attention_exact.py tests/test_gpu_classify.py tests/test_gpu_rows_sampling.py > gpurun_out/r6u_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --steps 64 > gpurun_out/r6u_bench_ov.json 2> gpurun_out/r6u_bench_ov.err || exit 1
BS_ATTN_OVERLAP=0 timeout -k 10 300 python bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --steps 64 > gpurun_out/r6u_bench_noov.json 2> gpurun_out/r6u_bench_noov.err || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --steps 64 > gpurun_out/r6u_bench_ov2.json 2>> gpurun_out/r6u_bench_ov.err || exit 1
