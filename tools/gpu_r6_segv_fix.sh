#!/bin/bash
# The round-5/6 SIGSEGV under rocprofv3 --pmc (gpurun_out/r6_segv.err): the same command with every decode step
# launched eagerly (BS_GRAPHS=0: no hipGraph replays), progress lines on.
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp BS_PROGRESS=1 BS_GRAPHS=0
rm -rf $R/gpurun_out/r6_segv2
cd /tmp && timeout -k 10 840 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/r6_segv2 \
  -o pmc --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --no-pmc --no-profile --steps 4 --warmup 1 \
  > $R/gpurun_out/r6_segv2.json 2> $R/gpurun_out/r6_segv2.err
rc=$?
echo "rocprofv3 rc $rc" >> $R/gpurun_out/r6_segv2.err
cd $R && find gpurun_out/r6_segv2 -name "*.csv" -size +20M -delete
grep -v "^\[bs_forward\]" gpurun_out/r6_segv2.err | tail -12
grep pipeline_bench gpurun_out/r6_segv2.err | tail -3
exit $rc
