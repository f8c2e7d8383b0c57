#!/bin/bash
# Round-end check of this tree: GPU tests, smoke(), default bench line, kernel-trace stats of the bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/final_prof -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc > $GRAFT_REPO_ROOT/gpurun_out/final_prof.log 2>&1
# batch-32 decode kernel mix (bloom-1b1, prompt 128)
cd $GRAFT_REPO_ROOT && bash tools/gpu_b32_prof.sh || exit 1
