#!/bin/bash
# C4 measurement: the bench line, a rocprofv3 kernel-trace/stats pass, then the PMC HBM bytes
# (FETCH_SIZE and WRITE_SIZE in separate passes), each step under its own time limit.
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4prof -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/c4prof_bench.json 2> $R/gpurun_out/c4prof_bench.log || exit $?
cd $R && CFG=c4 scripts/gpu/pmc_cfg.sh
