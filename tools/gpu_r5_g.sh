#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5g_pmc -o pmc --output-format csv -- $GRAFT_REPO_ROOT/tools/attn_prefill_bench > $GRAFT_REPO_ROOT/gpurun_out/r5g_pmc.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/pmc_mfma.py gpurun_out/r5g_pmc > gpurun_out/r5g_mfma_util.txt 2>&1
find gpurun_out/r5g_pmc -name "*.csv" -size +20M -delete
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5g_kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 4 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r5g_kt.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find gpurun_out/r5g_kt -name "*kernel_trace.csv" -delete
