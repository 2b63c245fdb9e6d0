#!/bin/bash
# Bench lines for the other BASELINE configs on one GPU (c3 at N=1: the scaling curve's own
# single-GPU point; c5: singleton-heavy).  Each step under its own time limit.
mkdir -p gpurun_out
for c in ${CONFIGS:-c3 c5}; do
  timeout -k 10 500 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.log || exit $?
done
