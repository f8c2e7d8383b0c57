# A/B of an env switch on the headline bench: bash tools/gpu_ab.sh NAME "ENV_A" "ENV_B" [bench args]
# writes gpurun_out/ab_NAME.log (tokens/s per arm, two runs each, alternating)
mkdir -p gpurun_out
name=$1; a=$2; b=$3; shift 3
out=gpurun_out/ab_$name.log; : > $out
for i in 1 2; do
  for arm in "$a" "$b"; do
    r=$(env $arm timeout -k 10 200 python -u bench.py --cpu-baseline 0 --no-pmc --no-profile "$@" 2>/dev/null | tail -1) || exit 1
    v=$(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f tok/s %.4f ms/step" % (d["value"], d["ms_per_step"]))')
    echo "[$arm] $* : $v" >> $out
  done
done
cat $out
