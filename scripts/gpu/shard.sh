#!/bin/bash
# sharded-path parity (LocalComm + the two-process CLI), the C3 full-size case, the function-level ABI
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_function_abi.py "tests/test_gpu_fullsize.py::test_fullsize_matches_oracle[c3_sharded8]" -m gpu -x -v -s --timeout 900 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/shard.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/shard.log; exit $rc
