#!/bin/bash
# rocprofv3 kernel trace of a short C2 bench run, split per read_bam pass (scripts/kernel_passes.py)
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ktrace -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/ktrace_bench.json 2> $R/gpurun_out/ktrace_bench.log || exit $?
cd $R && python3 scripts/kernel_passes.py "gpurun_out/ktrace/**/run_kernel_trace.csv" 5 gpurun_out/passes.json > gpurun_out/passes.txt
