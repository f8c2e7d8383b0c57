#!/bin/bash
# Round 4: prefill attention on the S^T layout (P from registers): its bench, the prefill parity tests, then the
# decode attention split A/B (64-position chunks per split) on the default bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
export BS_PARITY_LOG=$PWD/gpurun_out/ra_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 120 ./tools/attn_prefill_bench > gpurun_out/ra_attn_prefill.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_7b1_width.py tests/test_gpu_prefill_split.py tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ra_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ra_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_attn_split_ab.sh
