#!/bin/bash
# kernel traces of batched decode (bloom-1b1 B = 8, bloom-560m B = 8) and the B = 1 headline, per (kernel, grid)
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "bloom-1b1 8 128" "bloom-560m 8 16" "bloom-1b1 1 512"; do
  set -- $cfg
  tag=r5j_${1}_b$2
  cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$tag -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model $1 --batch $2 --prompt $3 --steps 32 --warmup 4 --cpu-baseline 0 --no-pmc --no-profile --no-pipeline-n1 --no-configs > $GRAFT_REPO_ROOT/gpurun_out/$tag.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT && python3 tools/trace_by_grid.py gpurun_out/$tag > gpurun_out/${tag}_by_grid.txt 2>&1
  find gpurun_out/$tag -name "*kernel_trace.csv" -delete
done
