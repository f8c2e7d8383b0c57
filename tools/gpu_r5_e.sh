#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/attn_stamps 2 1 > gpurun_out/r5e_stamps.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/attn_stamps 2 2 >> gpurun_out/r5e_stamps.txt 2>&1 || exit 1
timeout -k 10 200 ./tools/attn_prefill_bench > gpurun_out/r5e_attn.txt 2>&1 || exit 1
