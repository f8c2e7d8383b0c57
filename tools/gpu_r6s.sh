#!/bin/bash
# Kernel trace of a bloom-7b1 batch-16 decode (prompt 256; one configs[4] micro-batch at N = 1): per-kernel averages
# of the decode steps by (kernel, grid).
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/b16
cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/b16 -o b16 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model bloom-7b1 --batch 16 --prompt 256 --steps 32 --warmup 4 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 > $GRAFT_REPO_ROOT/gpurun_out/b16.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/trace_by_grid.py gpurun_out/b16 > gpurun_out/b16_by_grid.txt 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/b16 -name "*kernel_trace.csv" -delete
