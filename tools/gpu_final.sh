#!/bin/bash
# Round-end check of this tree: GPU tests, smoke(), default bench line, kernel-trace stats of the bench, batch-32
# kernel mix.  Kernel-trace CSVs are reduced to their summaries and deleted (gpurun copies back <= 64 MiB).
mkdir -p gpurun_out
export TMPDIR=/tmp
export BS_PARITY_LOG=$PWD/gpurun_out/final_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/final_prof -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc --no-pipeline-n1 > $GRAFT_REPO_ROOT/gpurun_out/final_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find gpurun_out/final_prof -name "*kernel_trace.csv" -delete
bash tools/gpu_b32_prof.sh || exit 1
find gpurun_out/b32 -name "*kernel_trace.csv" -delete
du -sh gpurun_out
