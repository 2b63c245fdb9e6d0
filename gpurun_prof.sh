#!/bin/bash
# full-size bench (default args) then a rocprofv3 kernel-trace/stats pass of the same workload
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${PROF_ARGS} > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.log
