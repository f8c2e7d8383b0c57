# MFMA utilisation counters of the headline prefill (rocprofv3 --pmc, own pass)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_mfma -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 4 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc_mfma.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/pmc_mfma.py gpurun_out/pmc_mfma > gpurun_out/pmc_mfma.txt
