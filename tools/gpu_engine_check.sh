#!/bin/bash
# Decode engine: in-kernel timeline, its GPU tests, then a short bench line.  Each step time-limited.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/engine_timeline 580 > gpurun_out/eng_timeline.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -v -x --timeout 120 --timeout-method thread "$@" > gpurun_out/eng_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/eng_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --engine 1 --no-pmc --cpu-baseline 0 > gpurun_out/eng_bench.json 2> gpurun_out/eng_bench.err || exit 1
