#!/bin/bash
# Round-4 check: batched-decode / 7b1-width / serve parity tests (fused LayerNorm statistics; logits vs the
# float64 checker; admission prefill), the product-pipeline tests (7b1 8-stage split, B=32 2-stage), serve
# tokens/s by prompt length, then one default bench line (pipeline_n1 with configs[3] / configs[4]).
mkdir -p gpurun_out
export TMPDIR=/tmp
export BS_PARITY_LOG=$PWD/gpurun_out/r4_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests/test_gpu_batched_gemv.py tests/test_gpu_7b1_width.py tests/test_gpu_parity.py -k "batched or 7b1 or width or serve" -v --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_batched.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4_pytest_batched.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_pipeline_7b1.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r4_pytest_7b1pipe.log 2>&1
rc2=$?; echo "pytest rc=$rc2" >> gpurun_out/r4_pytest_7b1pipe.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
./tools/gpu_serve_prompts.sh || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err
echo "bench rc=$?" >> gpurun_out/r4_bench.err
exit $rc
