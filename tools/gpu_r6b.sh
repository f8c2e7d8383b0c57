#!/bin/bash
# Round-6 pass 2: the new / re-bounded tests, the smoke, then one rocprofv3 --pmc run of the command that faulted in
# round 5 (gpurun_out/r5f_pmc.log) with bs_forward's call markers on (BS_TRACE_CALLS=1).
mkdir -p gpurun_out
R=$PWD
export BS_PARITY_LOG=$R/gpurun_out/r6b_parity_errors.jsonl
rm -f $BS_PARITY_LOG
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_attention_exact.py tests/test_gpu_parity.py tests/test_gpu_full_size.py \
  "tests/test_gpu_batched_gemv.py::test_small_batch_decode_middle_stage_widths" -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r6b_tests.log 2>&1
echo "pytest rc $?" >> gpurun_out/r6b_tests.log
[ -n "$SKIP_TESTS" ] || timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6b_smoke.log 2>&1 || exit 1
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 ./tools/attn_prefill_bench > gpurun_out/r6b_attn_prefill_ab.txt 2>&1 || exit 1
export TMPDIR=/tmp
export BS_TRACE_CALLS=1
export BS_DUMP_MAPS=$R/gpurun_out/r6_segv_maps.txt
rm -rf $R/gpurun_out/r6_segv
cd /tmp && timeout -k 10 500 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/r6_segv \
  -o pmc --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 4 --warmup 1 \
  > $R/gpurun_out/r6_segv.json 2> $R/gpurun_out/r6_segv.err
rc=$?
echo "rocprofv3 rc $rc" >> $R/gpurun_out/r6_segv.err
cd $R && find gpurun_out/r6_segv -name "*.csv" -size +20M -delete
tail -c 3000 gpurun_out/r6_segv.err | grep -v "^\[bs_forward\]" | tail -20
grep -c "^\[bs_forward\]" gpurun_out/r6_segv.err
tail -3 gpurun_out/r6b_tests.log
