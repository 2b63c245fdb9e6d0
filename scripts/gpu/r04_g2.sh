set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_function_abi.py > gpurun_out/r04_fabi_tests.log 2>&1 && \
CC_BENCH_DEVICES=1 timeout -k 10 900 python bench.py --gpus 2 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r04_c3_rehearse2_25m_bench.json 2> gpurun_out/r04_c3_rehearse2_25m_bench.log
