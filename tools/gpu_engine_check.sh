#!/bin/bash
# Decode engine: parity tests, then bench A/B (engine on / off, same box), each step time-limited.
mkdir -p gpurun_out
export TMPDIR=/tmp
export BS_PARITY_LOG=$PWD/gpurun_out/r4e_parity_errors.jsonl
rm -f $BS_PARITY_LOG
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -v -x --timeout 120 --timeout-method thread > gpurun_out/r4e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r4e_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for V in d8 d12 d4 thin2; do
  echo "== $V" >> gpurun_out/r4e_timeline.txt
  timeout -k 10 60 ./tools/engine_timeline_$V 580 >> gpurun_out/r4e_timeline.txt 2>&1 || exit 1
done
for E in 1 0 1 0; do
  timeout -k 10 200 python bench.py --steps 64 --warmup 8 --engine $E --no-pipeline-n1 --cpu-baseline 0 --no-pmc > gpurun_out/r4e_bench_$E.json 2>>gpurun_out/r4e_bench.err || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/r4e_bench_$E.json').read()); print('engine $E', r['value'], r['ms_per_step'], r['stage_hbm']['frac_of_peak'])" >> gpurun_out/r4e_ab.txt
done
exit $rc
