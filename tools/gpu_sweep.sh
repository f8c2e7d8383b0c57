# Sweep env settings on one bench configuration: bash tools/gpu_sweep.sh NAME "BENCH ARGS" "ENV1" "ENV2" ...
# writes gpurun_out/sweep_NAME.log (tokens/s per setting)
mkdir -p gpurun_out
name=$1; args=$2; shift 2
out=gpurun_out/sweep_$name.log; : > $out
for arm in "$@"; do
  r=$(env $arm timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --no-profile $args 2>/dev/null | tail -1) || exit 1
  v=$(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f tok/s %.4f ms/step" % (d["value"], d["ms_per_step"]))')
  echo "[$arm] $args : $v" >> $out
done
cat $out
