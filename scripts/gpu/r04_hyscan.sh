set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/hyscan
mkdir -p $O
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > $O/c5_new.json 2> $O/c5_new.log && \
CC_SCAN1=0 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > $O/c5_old.json 2> $O/c5_old.log && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_new.json 2> $O/c2_new.log && \
CC_SCAN1=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_old.json 2> $O/c2_old.log && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
