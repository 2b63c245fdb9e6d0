#!/bin/bash
# parity tests, then full-size bench + rocprofv3 (stops at the first failure/crash)
mkdir -p gpurun_out
timeout -k 10 800 python -m pytest tests -m gpu -q --tb=short > gpurun_out/tests.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
./gpurun_prof.sh
