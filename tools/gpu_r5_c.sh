#!/bin/bash
# prefill attention A/B + the prefill parity tests + rows8 batched decode tests + bench matrix batched rows
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/attn_prefill_bench > gpurun_out/r5c_attn.txt 2>&1 || exit 1
export BS_PARITY_LOG=$PWD/gpurun_out/r5c_parity.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill_split.py tests/test_gpu_parity.py tests/test_gpu_7b1_width.py tests/test_gpu_batched_gemv.py -k "prefill or tiny or split or family or golden or batched or rows8" > gpurun_out/r5c_pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_matrix.py --rows batched > gpurun_out/r5c_matrix.txt 2>&1
