#!/bin/bash
# The N-rank bench path on a one-GPU box: bench.py --gpus 2 spawns two ranks (torch.distributed.run),
# both on GPU 0 with gloo for the reduction (CC_BENCH_DEVICES=1), C3 blocks of 500 k pairs each.
mkdir -p gpurun_out
CC_BENCH_DEVICES=1 timeout -k 10 600 python bench.py --gpus 2 --pairs 500000 --steps 2 --warmup 1 --profile-steps 1 \
  --no-cpu-baseline > gpurun_out/bench_rehearse2.json 2> gpurun_out/bench_rehearse2.log
