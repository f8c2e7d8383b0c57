mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_int8.log 2>&1 || exit 1
out=gpurun_out/int8_batched.log; : > $out
for m in bloom-7b1 bloom-3b; do for b in 16 32; do for wt in int8 bf16; do
  r=$(timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-pmc --no-profile --model $m --batch $b --prompt 128 --weights $wt --steps 32 --warmup 4 2>/dev/null | tail -1) || exit 1
  echo "$m B=$b $wt: $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f tok/s %.3f ms/step" % (d["value"], d["ms_per_step"]))')" >> $out
done; done; done
cat $out
