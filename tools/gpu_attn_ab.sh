# decode attention 8 waves x 32 positions vs 4 waves x 64 (BS_ATTN_CH64=1): tests + bench A/B x2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  BS_ATTN_CH64=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_att64_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_att32_$rep.log 2>&1 || exit $?
done
BS_ATTN_CH64=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --model bloom-7b1 > gpurun_out/bench_att64_7b1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --model bloom-7b1 > gpurun_out/bench_att32_7b1.log 2>&1 || exit $?
