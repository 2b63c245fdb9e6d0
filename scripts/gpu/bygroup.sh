#!/bin/bash
# The deep tag sort keyed group-major on KB key bits (CC_DEEP_KEYBITS, default 48): the C4 oracle cases, then the C4 bench.
mkdir -p gpurun_out
export CC_DEEP_KEYBITS=${KB:-48}
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c4" > gpurun_out/tests_bg.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/tests_bg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4_bg.json 2> gpurun_out/bench_c4_bg.log || exit $?
