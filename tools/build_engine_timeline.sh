#!/bin/bash
# Builds the decode-engine timeline diagnostics (tools/engine_timeline.hip) in the A/B variants that
# profiles/r04_engine_timeline_ab.txt records (each binary run on the box as
# `./tools/engine_timeline_<variant>`): slots in flight 8 / 4 / 12, and the loader thinned to 1 / 2 slots in
# flight while its CU's gather wave sweeps.
set -e
cd "$(dirname "$0")/.."
F="hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/engine_timeline.hip"
pids=()
$F -o tools/engine_timeline_d8 & pids+=($!)
$F -DBS_ENGINE_D=4 -o tools/engine_timeline_d4 & pids+=($!)
$F -DBS_ENGINE_D=12 -o tools/engine_timeline_d12 & pids+=($!)
$F -DBS_ENGINE_THIN=1 -o tools/engine_timeline_thin1 & pids+=($!)
$F -DBS_ENGINE_THIN=2 -o tools/engine_timeline_thin2 & pids+=($!)
for p in "${pids[@]}"; do wait $p; done
