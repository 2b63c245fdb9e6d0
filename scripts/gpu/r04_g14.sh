set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_deep_rank.py tests/test_gpu_medium.py > gpurun_out/r04_g14_tests.log 2>&1 && \
CCAMD_LIB=build/var/dfprof/libccamd.so timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 --profile-steps 1 > gpurun_out/r04_g14_c4prof.json 2> gpurun_out/r04_g14_c4prof.log && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_g14_alltests.log 2>&1
