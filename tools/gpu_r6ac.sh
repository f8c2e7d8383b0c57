#!/bin/bash
# Round 6: the batched tile GEMV with four m-tiles (33 <= M <= 64 tokens): parity, then the classification passes of
# bloom-1b1 at 64 tokens (serve.py --max-length 0, one sample a pass) profiled with the old dispatch
# (BS_TILES_MAX_M=32: the prefill GEMMs) and the new one.
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_batched_gemv.py tests/test_gpu_prefill_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6ac_tests.log 2>&1 || { tail -30 gpurun_out/r6ac_tests.log; exit 1; }
tail -2 gpurun_out/r6ac_tests.log
for mm in 32 64; do
  export BS_TILES_MAX_M=$mm
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6ac_m$mm -o run --output-format csv -- \
      python3 -m distributed_inference_demo_amd.serve --model bloom-1b1 --max-length 0 --n-labels 2 --num-sample 64 \
      --prompt-len 64 --core-pool-size 1 > $GRAFT_REPO_ROOT/gpurun_out/r6ac_m$mm.log 2>&1 ) || exit 1
  find gpurun_out/r6ac_m$mm -name "*kernel_trace.csv" -delete
  for pool in 1 4; do
    timeout -k 10 120 python -u -m distributed_inference_demo_amd.serve --model bloom-1b1 --max-length 0 --n-labels 2 \
      --num-sample 256 --prompt-len 48 --core-pool-size $pool > gpurun_out/r6ac_serve_m${mm}_p$pool.log 2>&1 || exit 1
    tail -1 gpurun_out/r6ac_serve_m${mm}_p$pool.log | cut -c1-60
  done
done
