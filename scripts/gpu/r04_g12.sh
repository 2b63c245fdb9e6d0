set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CC_DEEP_FAM=1 CCAMD_LIB=build/var/dfprof/libccamd.so timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 --profile-steps 1 > gpurun_out/r04_g12_c4prof.json 2> gpurun_out/r04_g12_c4prof.log && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deep_rank.py tests/test_gpu_golden.py tests/test_gpu_deferred.py tests/test_gpu_large.py > gpurun_out/r04_g12_tests.log 2>&1
