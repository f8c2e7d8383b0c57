#!/bin/bash
# Round-3 check: the whole GPU suite (new 7b1-width / nccl world-1 / stream-switch tests included),
# smoke(), then one default bench line.  Each GPU step has its own time limit; a failure ends the call.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/r3_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
echo "bench rc=$?" >> gpurun_out/r3_bench.err
exit $rc
