#!/bin/bash
# Round-end measurement: smoke, the GPU suite, the c2 bench with rocprof + PMC (prof.sh), c4.
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || exit $?
PMC=1 scripts/gpu/prof.sh || exit $?
CONFIGS=c4 scripts/gpu/configs.sh || exit $?
