#!/bin/bash
# GPU parity tests, then the scope PMC passes + bench (gpurun_pmcbench.sh), then a
# rocprofv3 --kernel-trace --stats pass of the same bench.
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || exit $?
./gpurun_pmcbench.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.log
