#!/bin/bash
# Round 5 checkpoint: full GPU suite (parity log), parity-study device phase, bench line, MFMA-busy PMC pass
mkdir -p gpurun_out
export TMPDIR=/tmp
export BS_PARITY_LOG=$PWD/gpurun_out/r5f_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5f_pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/parity_study.py gpu --layers 2,30 --tag tr > gpurun_out/r5f_study.log 2>&1 || exit 1
timeout -k 10 200 python tools/parity_study.py gpu --layers 2 --batch 32 --tag tr >> gpurun_out/r5f_study.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5f_pmc -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 4 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r5f_pmc.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/pmc_mfma.py gpurun_out/r5f_pmc > gpurun_out/r5f_mfma_util.txt 2>&1; find gpurun_out/r5f_pmc -name "*.csv" -size +20M -delete
