set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_extract_barcodes.py tests/test_gpu_debug_bounds.py tests/test_gpu_function_abi.py tests/test_gpu_golden.py tests/test_gpu_shard.py > gpurun_out/r04_g6_tests.log 2>&1 && \
CCIO_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --profile-steps 1 > gpurun_out/r04_g6_c2.json 2> gpurun_out/r04_g6_c2.log
