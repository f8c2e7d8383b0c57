# GEMV probe + parity tests + bench (+ optional rocprof) in one GPU call.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 ./tools/gemv_probe > gpurun_out/gemv_probe.log 2>&1 || exit $?
PROF=${PROF:-0} bash tools/gpu_round.sh
