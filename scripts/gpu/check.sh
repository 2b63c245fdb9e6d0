#!/bin/bash
# the whole GPU suite, then the C2 bench and its per-pass kernel breakdown
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 1500 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/tests.log 2>&1; rc=$?; echo "EXIT $rc" >> gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit $?
scripts/gpu/passes.sh
