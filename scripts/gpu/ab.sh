mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_vote.py tests/test_gpu_large.py -x -q --timeout 280 --timeout-method thread > gpurun_out/tests_ab.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_u2.json 2> gpurun_out/ab_u2.log || exit 1
CCAMD_LIB=$PWD/scratch_libs/libccamd_u4.so timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_u4.json 2> gpurun_out/ab_u4.log || exit 1
