#!/bin/bash
# C2 bench (host breakdown of the end-to-end pass), then the C4 bench and its rocprofv3 kernel
# stats (per-kernel totals of a short run).  Each GPU step under its own time limit.
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit $?
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4prof -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/c4prof_bench.json 2> $R/gpurun_out/c4prof_bench.log || exit $?
