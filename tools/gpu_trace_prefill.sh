# kernel trace of the bench (prefill + decode), per (kernel, grid) averages: bash tools/gpu_trace_prefill.sh NAME [env...]
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; shift
cd /tmp && env "$@" timeout -s KILL 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tr_$name -o tr --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/tr_$name.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/trace_by_grid.py gpurun_out/tr_$name gemm > gpurun_out/tr_$name.txt; python3 tools/trace_by_grid.py gpurun_out/tr_$name attn_prefill >> gpurun_out/tr_$name.txt; cat gpurun_out/tr_$name.txt
