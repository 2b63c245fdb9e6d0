#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_function_abi.py tests/test_known_answers.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/abi.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/abi.log; exit $rc
