# PMC counters of the prefill GEMMs, one rocprofv3 --pmc pass per counter set, for the arms given as
# env strings: [PMC_FILE=sets.txt] bash tools/gpu_pmc_gemm.sh "BS_GEMM_XCD=1" "BS_GEMM_XCD=0"
# PMC_FILE: one counter set per line, counters separated by commas (default: hit rate / SQ / TA sets).
mkdir -p gpurun_out
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_gemm.txt; : > $out
if [ -n "$PMC_FILE" ]; then mapfile -t sets < <(tr ',' ' ' < "$PMC_FILE"); else
  sets=("TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
        "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
        "TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"); fi
i=0
for arm in "$@"; do
  for set in "${sets[@]}"; do
    [ -z "$set" ] && continue
    i=$((i+1))
    cd /tmp && env $arm timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmcg$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/pmcg$i.log 2>&1 || exit 1
    cd $GRAFT_REPO_ROOT && { echo "== [$arm] $set"; python3 tools/pmc_table.py gpurun_out/pmcg$i gemm_mfma2; } >> $out
  done
done
cat $out
