# decode sweeps on bloom-1b1 B=1: plain rows per wave (BS_PLAIN_R), attention splits (BS_ATTN_SPLITS)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 96 "$@"; }
run > gpurun_out/dsw_base.log 2>&1 || exit $?
for r in 1 2 4; do BS_PLAIN_R=$r run > gpurun_out/dsw_r$r.log 2>&1 || exit $?; done
for n in 1 2 4; do BS_ATTN_SPLITS=$n run > gpurun_out/dsw_s$n.log 2>&1 || exit $?; done
run > gpurun_out/dsw_base2.log 2>&1 || exit $?
