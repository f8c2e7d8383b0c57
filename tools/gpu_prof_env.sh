# kernel-trace stats of the headline bench under an env setting: bash tools/gpu_prof_env.sh NAME "ENV" [bench args]
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; e=$2; shift 2
env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- python3 bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 40 --warmup 4 "$@" > gpurun_out/prof_$name.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$name -name '*kernel_stats.csv' | head -1)
python3 - "$f" > gpurun_out/prof_$name.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:90]:90s} {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us  total {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
cat gpurun_out/prof_$name.txt
