#!/bin/bash
# Round 4: batched decode rows (gemv_ldsw4 ring depth 3 at bloom-1b1 widths), then the default bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_matrix.py --rows batched > gpurun_out/r4d_matrix.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_bench.err || exit 1
