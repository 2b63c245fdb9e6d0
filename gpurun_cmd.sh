#!/bin/bash
# one GPU call: parity tests, then (unless a crash/fault) a short bench
mkdir -p gpurun_out
timeout -k 10 800 python -m pytest tests -m gpu -q --tb=short > gpurun_out/tests.log 2>&1
rc=$?
echo "EXIT $rc" >> gpurun_out/tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --pairs ${BENCH_PAIRS:-300000} --steps 3 --warmup 1 ${BENCH_EXTRA} > gpurun_out/bench.json 2> gpurun_out/bench.log
rc=$?
echo "EXIT $rc" >> gpurun_out/bench.log
exit $rc
