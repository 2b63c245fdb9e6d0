set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deep_rank.py tests/test_gpu_vote.py tests/test_gpu_large.py tests/test_gpu_golden.py tests/test_gpu_medium.py > gpurun_out/r04_g21_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 5 --profile-steps 1 > gpurun_out/r04_g21_c4.json 2> gpurun_out/r04_g21_c4.log
