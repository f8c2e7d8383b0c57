#!/bin/bash
# Round-6 evidence pass 3: the whole GPU suite (every bf16 check's error recorded), smoke, the default bench line,
# and the N = 8 middle rank's host enqueue with its RCCL pairs (tools/host_enqueue.py).
mkdir -p gpurun_out
R=$PWD
export BS_PARITY_LOG=$R/gpurun_out/r6c_parity_errors.jsonl BS_PROGRESS=1
rm -f $BS_PARITY_LOG
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6c_tests.log 2>&1 || { tail -30 gpurun_out/r6c_tests.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r6c_bench.json 2> gpurun_out/r6c_bench.err || exit 1
timeout -k 10 300 python tools/host_enqueue.py > gpurun_out/r6c_host_enqueue.json 2> gpurun_out/r6c_host_enqueue.err || exit 1
tail -2 gpurun_out/r6c_tests.log; cat gpurun_out/r6c_smoke.log; cut -c1-400 gpurun_out/r6c_bench.json; cat gpurun_out/r6c_host_enqueue.json
