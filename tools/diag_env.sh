mkdir -p gpurun_out
export DIAG_SWEEP=1 DIAG_DTYPES=bf16 DIAG_DIMS=4096x32,3072x24,3584x28,4096x128
for v in "" "BS_GEMV_MFMA=1" "BS_GEMV_TILES_OFF=1" "BS_GEMV_MFMA=1 BS_GEMV_TILES_OFF=1"; do
  echo "=== env: $v" >> gpurun_out/diag_env.log
  env $v timeout -k 10 200 python -u tools/diag_parity.py >> gpurun_out/diag_env.log 2>&1 || exit 1
done
