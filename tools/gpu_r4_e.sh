#!/bin/bash
# Round 4: GEMM dispatch at long-prompt shapes (>= 512 tiles: 2-stage / two blocks per CU vs 3-stage), then the
# prefill MFMA utilisation counters (own PMC pass).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/gemm_splitk_bench > gpurun_out/re_b2b.txt 2>&1 || exit 1
bash tools/gpu_pmc_mfma.sh || exit 1
