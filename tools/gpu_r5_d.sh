#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 ./tools/attn_prefill_bench > gpurun_out/r5d_attn.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/rows8_bench > gpurun_out/r5d_rows8.txt 2>&1 || exit 1
