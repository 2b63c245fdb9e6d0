set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 10 --profile-steps 1"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vote.py tests/test_gpu_golden.py tests/test_gpu_function_abi.py tests/test_gpu_deferred.py tests/test_gpu_medium.py > gpurun_out/r04_g5_tests.log 2>&1 && \
timeout -k 10 300 $B > gpurun_out/r04_g5_new.json 2> gpurun_out/r04_g5_new.log && \
CCAMD_LIB=build/var/base/libccamd.so timeout -k 10 300 $B > gpurun_out/r04_g5_base.json 2> gpurun_out/r04_g5_base.log && \
CCAMD_LIB=build/var/v8/libccamd.so timeout -k 10 300 $B > gpurun_out/r04_g5_v8.json 2> gpurun_out/r04_g5_v8.log && \
CCAMD_LIB=build/var/v7/libccamd.so timeout -k 10 300 $B > gpurun_out/r04_g5_v7.json 2> gpurun_out/r04_g5_v7.log
