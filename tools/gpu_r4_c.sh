#!/bin/bash
# Round 4: GEMM dispatch A/B (XCD-aware placement) first, then the whole GPU suite.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 ./tools/gemm_splitk_bench > gpurun_out/gemm_b2b_xm.txt 2>&1 || exit 1
export BS_PARITY_LOG=$PWD/gpurun_out/parity_errors.jsonl
rm -f $BS_PARITY_LOG
bash tools/gpu_tests.sh
