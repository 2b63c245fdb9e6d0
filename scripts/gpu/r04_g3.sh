set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r04_g3_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r04_g3_c2_bench.json 2> gpurun_out/r04_g3_c2_bench.log && \
CC_BENCH_DEVICES=1 timeout -k 10 900 python bench.py --gpus 2 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r04_g3_rehearse2_bench.json 2> gpurun_out/r04_g3_rehearse2_bench.log
