#!/bin/bash
# The full-size parity suite (tests/test_gpu_fullsize.py) plus the sharded tests, with progress lines.
mkdir -p gpurun_out
timeout -k 10 1300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_shard.py -m gpu -x -v -s --timeout 1500 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/fullsize.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/fullsize.log; exit $rc
