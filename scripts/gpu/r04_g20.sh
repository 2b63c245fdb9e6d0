set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_g20_tests.log 2>&1 && \
CCIO_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --profile-steps 1 > gpurun_out/r04_g20_c2.json 2> gpurun_out/r04_g20_c2.log && \
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 5 --profile-steps 1 > gpurun_out/r04_g20_c4.json 2> gpurun_out/r04_g20_c4.log && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --profile-steps 1 > gpurun_out/r04_g20_c5.json 2> gpurun_out/r04_g20_c5.log
