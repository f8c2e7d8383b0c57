#!/bin/bash
# MFMA busy per (shape, variant) of the prefill attention bench (one PMC pass)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5u_pmc -o pmc --output-format csv -- $GRAFT_REPO_ROOT/tools/attn_prefill_bench > $GRAFT_REPO_ROOT/gpurun_out/r5u_pmc.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/pmc_mfma_seq.py gpurun_out/r5u_pmc gpurun_out/r5u_pmc.log > gpurun_out/r5u_mfma_util.txt 2>&1
find gpurun_out/r5u_pmc -name "*.csv" -size +20M -delete
