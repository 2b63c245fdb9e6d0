#!/bin/bash
# Parity tests (GPU), then the SSCS-stage variant timings of gpurun_vote.sh.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/tests.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
./gpurun_vote.sh
