#!/bin/bash
# The N-rank bench path on a one-GPU box: bench.py --gpus N spawns N ranks (torch.distributed.run),
# all on GPU 0 with gloo for the reduction (CC_BENCH_DEVICES=1), C3 blocks (PAIRS per rank; default
# the full 10 M pairs per rank).
mkdir -p gpurun_out
N=${N:-2}
ARGS="--gpus $N --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline"
if [ -n "$PAIRS" ]; then ARGS="$ARGS --pairs $PAIRS"; fi
CC_BENCH_DEVICES=1 timeout -k 10 900 python bench.py $ARGS > gpurun_out/bench_rehearse$N.json 2> gpurun_out/bench_rehearse$N.log
