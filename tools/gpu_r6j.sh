#!/bin/bash
# Round-6: the 256 x 256 prefill tiles -- the tests that run them (bitwise against the 128 x 128 path, the configs[4]
# pipeline schedule, the 7b1-width prefills), then the default bench line (configs4 prefill TFLOP/s).
mkdir -p gpurun_out
export BS_PARITY_LOG=$PWD/gpurun_out/r6j_parity_errors.jsonl BS_PROGRESS=1
rm -f $BS_PARITY_LOG
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefill_split.py tests/test_gpu_pipeline_7b1.py tests/test_gpu_7b1_width.py \
  tests/test_gpu_attention_exact.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6j_tests.log 2>&1 || { tail -30 gpurun_out/r6j_tests.log; exit 1; }
tail -2 gpurun_out/r6j_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r6j_bench.json 2> gpurun_out/r6j_bench.err || exit 1
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r6j_bench.json').read().strip().splitlines()[-1])
p=d['pipeline_n1']
print('headline', d['value'], 'prefill', d['prefill']['achieved_TFLOPs'])
for c,r in p['configs4']['by_ctx'].items(): print('configs4', c, r['value'], r['prefill']['achieved_TFLOPs'])
print('configs3', p['configs3']['value'], p['configs3']['prefill']['achieved_TFLOPs'])
PY
