#!/bin/bash
# One GPU call: parity tests, then the bench + rocprofv3 passes (prof.sh).  Every GPU step has its
# own time limit; the script stops at the first failure, crash or timeout.
# usage (repo root): scripts/gpu/all.sh      env: PYTEST_ARGS, BENCH_ARGS, PMC=1, SKIP_TESTS=1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/tests.log 2>&1
  rc=$?; echo "EXIT $rc" >> gpurun_out/tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
scripts/gpu/prof.sh
