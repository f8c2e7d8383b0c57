#!/bin/bash
# prefill attention key groups by shape: parity of the wide-head prefill tests + prefill tests
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_7b1_width.py tests/test_gpu_prefill_split.py > gpurun_out/r5n_prefill.log 2>&1 || exit 1
