#!/bin/bash
# Prefill GEMM study: K-step decomposition (tools/kstep_probe), then our dispatch vs hipBLASLt on the same box,
# both timed as 20 back-to-back launches between events.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/kstep_probe > gpurun_out/kstep_probe.txt 2>&1 || exit 1
timeout -k 10 200 ./tools/gemm_splitk_bench > gpurun_out/gemm_b2b.txt 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_shapes_torch.py > gpurun_out/gemm_hipblaslt.txt 2>&1 || exit 1
