#!/bin/bash
# The other configs' bench lines on the final build (C3 at one GPU, C5).
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || exit $?
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.log || exit $?
