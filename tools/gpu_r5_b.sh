#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/host_enqueue.py > gpurun_out/r5b_host_enqueue.json 2> gpurun_out/r5b_host_enqueue.err || exit 1
N_MB=8 timeout -k 10 200 python tools/host_enqueue.py >> gpurun_out/r5b_host_enqueue.json 2>> gpurun_out/r5b_host_enqueue.err || exit 1
timeout -k 10 400 python tools/parity_study.py gpu --layers 2,30 --tag lib > gpurun_out/r5b_study.log 2>&1 || exit 1
