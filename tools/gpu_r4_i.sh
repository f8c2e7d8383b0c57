#!/bin/bash
# Round 4 (informational): prefill GEMM grids at bloom-1b1 1024 / 2048 tokens.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/gemm_splitk_bench > gpurun_out/ri_b2b.txt 2>&1 || exit 1
