set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 10 --profile-steps 1"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vote.py tests/test_gpu_golden.py tests/test_gpu_function_abi.py > gpurun_out/r04_g4_tests.log 2>&1 && \
CCAMD_LIB=build/var/base/libccamd.so timeout -k 10 300 $B > gpurun_out/r04_g4_base.json 2> gpurun_out/r04_g4_base.log && \
timeout -k 10 300 $B > gpurun_out/r04_g4_new.json 2> gpurun_out/r04_g4_new.log && \
CC_SV_BLOCKS=0 timeout -k 10 300 $B > gpurun_out/r04_g4_nopersist.json 2> gpurun_out/r04_g4_nopersist.log && \
CC_SV_BLOCKS=2560 timeout -k 10 300 $B > gpurun_out/r04_g4_p2560.json 2> gpurun_out/r04_g4_p2560.log
