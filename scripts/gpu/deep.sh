#!/bin/bash
# Deep position groups (k_deep_qsort / k_deep_rank): the large oracle cases with deep groups, the
# deferred steps, then the C4 bench and its kernel stats.  Each GPU step under its own time limit.
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 700 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_deferred.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_deep.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests_deep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.log || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log || exit $?
if [ -n "$FULLSIZE" ]; then
  timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/fullsize.log 2>&1
  rc=$?; echo "EXIT $rc" >> gpurun_out/fullsize.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
