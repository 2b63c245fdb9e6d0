#!/bin/bash
# the rank-local test, then bench.py --gpus 2 rehearsed on this one GPU (both ranks on GPU 0, gloo)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -k rank_local -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ranklocal.log 2>&1 || exit $?
CC_BENCH_DEVICES=1 timeout -k 10 900 python bench.py --gpus 2 --steps 5 --warmup 1 ${BENCH_ARGS} > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log || exit $?
