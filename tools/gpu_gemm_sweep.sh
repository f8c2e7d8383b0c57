# prefill GEMM variant sweep on the bench's prefill numbers (one run per arm):
#   bash tools/gpu_gemm_sweep.sh NAME "ENV_1" "ENV_2" ... [-- bench args]
mkdir -p gpurun_out
name=$1; shift
arms=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done; [ "$1" = "--" ] && shift
out=gpurun_out/sweep_$name.log; : > $out
for arm in "${arms[@]}"; do
  r=$(env $arm timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --steps 8 --warmup 2 "$@" 2>/dev/null | tail -1) || exit 1
  v=$(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read())["prefill"]; print("prefill %.3f ms  gemm %.1f TFLOP/s (%.3f of peak)" % (d["ms"], d.get("gemm_TFLOPs", 0), d.get("gemm_frac_of_peak", 0)))')
  echo "[$arm] $* : $v" >> $out
done
cat $out
