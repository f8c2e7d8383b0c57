#!/bin/bash
# Round evidence without the test suite: smoke(), the default bench line (timed), kernel-trace stats of the bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/ev_smoke.log 2>&1 || exit 1
s=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/ev_bench.json 2> gpurun_out/ev_bench.err || exit 1
echo "bench wall $(( $(date +%s) - s )) s" >> gpurun_out/ev_bench.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ev_prof -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc > $GRAFT_REPO_ROOT/gpurun_out/ev_prof.log 2>&1
