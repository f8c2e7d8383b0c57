#!/bin/bash
# Round-6 evidence pass 1: the GPU suite (every bf16 check's error recorded, incl. the tight checks against the
# emulating checker), smoke, the h = 4096 hidden-state study (device side) and the fp32-reference study.
mkdir -p gpurun_out
export BS_PARITY_LOG=$PWD/gpurun_out/r6a_parity_errors.jsonl
rm -f $BS_PARITY_LOG gpurun_out/fp32ref_study.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6a_tests.log 2>&1
echo "pytest rc $?" >> gpurun_out/r6a_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a_smoke.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/parity_study_hidden.py gpu > gpurun_out/r6a_study_hidden.log 2>&1 || exit 1
timeout -k 10 420 python -u tools/fp32ref_study.py run --seeds 4 > gpurun_out/r6a_fp32ref.log 2>&1 || exit 1
tail -3 gpurun_out/r6a_tests.log
