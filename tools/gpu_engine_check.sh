#!/bin/bash
# The decode-engine experiment (tools/engine/engine.hip, not part of the library): in-kernel timelines of the
# A/B build variants (tools/build_engine_timeline.sh), each step time-limited.
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r4e_timeline.txt
for V in d8 d12 d4 thin2; do
  echo "== $V" >> gpurun_out/r4e_timeline.txt
  timeout -k 10 60 ./tools/engine_timeline_$V 580 >> gpurun_out/r4e_timeline.txt 2>&1 || exit 1
done
