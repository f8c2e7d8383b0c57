#!/bin/bash
# Attention-tail check: the parity suites that run batch-1 decode, then the headline bench with the tail on and off.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_attention_exact.py tests/test_gpu_classify.py > gpurun_out/r6t_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --steps 64 > gpurun_out/r6t_bench_tail.json 2> gpurun_out/r6t_bench_tail.err || exit 1
BS_ATTN_TAIL=0 timeout -k 10 300 python bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --steps 64 > gpurun_out/r6t_bench_notail.json 2> gpurun_out/r6t_bench_notail.err || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 --steps 64 > gpurun_out/r6t_bench_tail2.json 2>> gpurun_out/r6t_bench_tail.err || exit 1
