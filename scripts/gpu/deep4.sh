#!/bin/bash
# Deep position groups: the large oracle cases + deferred + golden, the C4 bench, its kernel stats.
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 700 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_deferred.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_deep.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests_deep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4prof -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/c4prof_bench.json 2> $R/gpurun_out/c4prof_bench.log || exit $?
