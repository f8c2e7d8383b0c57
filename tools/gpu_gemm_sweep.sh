# prefill GEMM tile sweep (BS_GEMM_TILE) on the bench workloads: 1b1 S=512 and 7b1 B=8 S=512
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 0 1 2 3 4; do
  BS_GEMM_TILE=$t timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --steps 8 --warmup 2 > gpurun_out/gemm_tile_$t.log 2>&1 || exit $?
  BS_GEMM_TILE=$t timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --steps 8 --warmup 2 --model bloom-7b1 --batch 8 > gpurun_out/gemm_tile_7b1_$t.log 2>&1 || exit $?
done
