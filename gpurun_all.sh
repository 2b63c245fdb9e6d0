#!/bin/bash
# One GPU call: parity tests, then the full-size bench + rocprofv3 passes (gpurun_prof.sh).
# Every GPU step has its own time limit; the script stops at the first failure, crash or timeout.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/tests.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
./gpurun_prof.sh
