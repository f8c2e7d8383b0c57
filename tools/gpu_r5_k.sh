#!/bin/bash
# batched GEMV geometry sweep + fused attention/dense A/B tool
mkdir -p gpurun_out
timeout -k 10 300 ./tools/attn_dense_fused > gpurun_out/r5k_attn_dense.txt 2>&1 || exit 1
timeout -k 10 600 ./tools/tiles_bench > gpurun_out/r5k_tiles.txt 2>&1 || exit 1
