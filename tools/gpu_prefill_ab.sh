# prefill GEMM A/B on the bench's prefill numbers: bash tools/gpu_prefill_ab.sh NAME "ENV_A" "ENV_B" [bench args]
mkdir -p gpurun_out
name=$1; a=$2; b=$3; shift 3
out=gpurun_out/pab_$name.log; : > $out
for i in 1 2; do
  for arm in "$a" "$b"; do
    r=$(env $arm timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --steps 16 --warmup 2 "$@" 2>/dev/null | tail -1) || exit 1
    v=$(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read())["prefill"]; print("prefill %.3f ms  gemm %.1f TFLOP/s (%.3f of peak)  all %.1f TFLOP/s" % (d["ms"], d.get("gemm_TFLOPs", 0), d.get("gemm_frac_of_peak", 0), d["achieved_TFLOPs"]))')
    echo "[$arm] $* : $v" >> $out
  done
done
cat $out
