set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scan1
O=gpurun_out/scan1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_bench.json 2> $O/c2_bench.log && \
CC_SCAN2=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_scan2_bench.json 2> $O/c2_scan2_bench.log && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > $O/c5_bench.json 2> $O/c5_bench.log && \
CC_SCAN2=1 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > $O/c5_scan2_bench.json 2> $O/c5_scan2_bench.log && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
