# evidence: smoke, default bench line, kernel trace, config matrix, HBM probe
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_evidence.sh || exit 1
timeout -k 10 900 python -u tools/bench_matrix.py > gpurun_out/matrix.log 2>&1 || exit 1
