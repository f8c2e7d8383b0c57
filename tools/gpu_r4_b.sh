#!/bin/bash
# Round-4 check B: the fused-LayerNorm paths again (stats kernel for a stage's first layer), the 7b1-width test
# with the measured checker-noise bound, the product-pipeline tests, and the batched decode bench rows.
mkdir -p gpurun_out
export TMPDIR=/tmp
export BS_PARITY_LOG=$PWD/gpurun_out/r4b_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests/test_gpu_batched_gemv.py tests/test_gpu_7b1_width.py tests/test_gpu_pipeline_7b1.py tests/test_gpu_parity.py -k "batched or 7b1 or width or serve or graph or split" -v --timeout 400 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4b_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python tools/bench_matrix.py --rows batched > gpurun_out/r4b_matrix.log 2>&1
echo "matrix rc=$?" >> gpurun_out/r4b_matrix.log
exit $rc
