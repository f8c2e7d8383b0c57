#!/bin/bash
# Round 5 first call: the default bench line (configs2 / replicas / scaling_ref under pipeline_n1) and the
# host-enqueue probe at the N = 8 stage shape.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || exit 1
timeout -k 10 200 python tools/host_enqueue.py > gpurun_out/r5a_host_enqueue.json 2> gpurun_out/r5a_host_enqueue.err || exit 1
N_MB=8 timeout -k 10 200 python tools/host_enqueue.py >> gpurun_out/r5a_host_enqueue.json 2>> gpurun_out/r5a_host_enqueue.err || exit 1
timeout -k 10 400 python tools/parity_study.py gpu --layers 2,30 --tag lib > gpurun_out/r5a_study.log 2>&1 || exit 1
