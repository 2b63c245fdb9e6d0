#!/bin/bash
# End-of-round call: the whole GPU suite, the C2 bench, then the C4 measurement (bench, rocprof,
# PMC).  Each step under its own time limit.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit $?
scripts/gpu/measure_c4.sh
