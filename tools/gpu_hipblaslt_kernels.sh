#!/bin/bash
# Which hipBLASLt kernels torch's F.linear runs on the prefill shapes (kernel names carry the macro tile / split).
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/hbl_prof -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/gemm_shapes_torch.py > $GRAFT_REPO_ROOT/gpurun_out/hbl_prof.log 2>&1
