set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ltab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deep_rank.py tests/test_gpu_engine_switches.py > $O/tests.log 2>&1 && \
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_new1.json 2> $O/c4_new1.log && \
CC_LTAB_SPARSE=1 timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_old.json 2> $O/c4_old.log && \
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_new2.json 2> $O/c4_new2.log
