#!/bin/bash
# Round measurement: smoke, the C2 bench (with the CPU baseline) + rocprofv3 kernel stats + PMC
# bytes (prof.sh), each step under its own time limit.
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
PMC=1 scripts/gpu/prof.sh || exit $?
