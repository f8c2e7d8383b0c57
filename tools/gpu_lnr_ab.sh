# LN-fused rows GEMV rows-per-wave thresholds (BS_LN_R2_MIN / BS_LN_R4_MIN), bench A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "4096 12288" "2048 12288" "4096 6144" "2048 4096"; do
  set -- $cfg
  BS_LN_R2_MIN=$1 BS_LN_R4_MIN=$2 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc > gpurun_out/bench_lnr_$1_$2.log 2>&1 || exit $?
  BS_LN_R2_MIN=$1 BS_LN_R4_MIN=$2 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --model bloom-560m > gpurun_out/bench_lnr_560m_$1_$2.log 2>&1 || exit $?
done
