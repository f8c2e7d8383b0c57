#!/bin/bash
# Round 4: one-wave-per-row LayerNorm (batched decode, prefill): the tests that reach it, the batched decode rows,
# the batch-32 kernel mix.
mkdir -p gpurun_out
export TMPDIR=/tmp
export BS_PARITY_LOG=$PWD/gpurun_out/rg_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 700 python -u -m pytest tests/test_gpu_batched_gemv.py tests/test_gpu_parity.py tests/test_gpu_prefill_split.py tests/test_gpu_7b1_width.py tests/test_gpu_pipeline.py tests/test_gpu_int8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rg_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/rg_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_matrix.py --rows batched > gpurun_out/rg_matrix.log 2>&1 || exit 1
bash tools/gpu_b32_prof.sh || exit 1
find gpurun_out/b32 -name "*kernel_trace.csv" -delete
