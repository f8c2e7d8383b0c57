#!/bin/bash
# Kernel trace of a bloom-1b1 batch-32 decode (prompt 128): per-kernel averages of the decode steps
# (kernel trace and stats, then a per-(kernel, grid) table).
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/b32
cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/b32 -o b32 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --batch 32 --prompt 128 --steps 32 --warmup 4 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 > $GRAFT_REPO_ROOT/gpurun_out/b32.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/trace_by_grid.py gpurun_out/b32 > gpurun_out/b32_by_grid.txt 2>&1
