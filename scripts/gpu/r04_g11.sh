set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CC_DEEP_FAM=1 CCAMD_LIB=build/var/dfprof/libccamd.so timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 --profile-steps 0 > gpurun_out/r04_g11_c4prof.json 2> gpurun_out/r04_g11_c4prof.log && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_g11_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > gpurun_out/r04_g11_c5.json 2> gpurun_out/r04_g11_c5.log && \
CCIO_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --profile-steps 1 > gpurun_out/r04_g11_c2.json 2> gpurun_out/r04_g11_c2.log
