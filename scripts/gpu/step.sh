#!/bin/bash
# One GPU call: the named test files first (TESTS), the C2 bench, then (FULL=1) the whole GPU suite.
# Each GPU step under its own time limit; stops at the first failure.
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_quick.log 2>&1
  rc=$?; echo "EXIT $rc" >> gpurun_out/tests_quick.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit $?
if [ -n "$FULL" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
  rc=$?; echo "EXIT $rc" >> gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
