#!/bin/bash
# A/B of engine builds on the c2 bench: the in-tree libccamd.so, then each scratch_libs/*.so
# (CCAMD_LIB), with AB_ARGS passed to bench.py.  Each run under its own time limit; stops at the first failure.
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab_base.json 2> gpurun_out/ab_base.log || exit 1
for so in scratch_libs/*.so; do
  n=$(basename $so .so)
  CCAMD_LIB=$PWD/$so timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.log || exit 1
done
