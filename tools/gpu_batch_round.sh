# Batched-GEMV probe + parity tests + bench in one GPU call.
mkdir -p gpurun_out
export TMPDIR=/tmp
PROBE_BATCH=1 timeout -k 10 200 ./tools/gemv_probe > gpurun_out/gemv_probe_batch.log 2>&1 || exit $?
bash tools/gpu_round.sh
