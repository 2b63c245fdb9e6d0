set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/csn
mkdir -p $O
B=build/var/base/libccamd.so
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_new1.json 2> $O/c2_new1.log && \
CCAMD_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_base1.json 2> $O/c2_base1.log && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_new2.json 2> $O/c2_new2.log && \
CCAMD_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_base2.json 2> $O/c2_base2.log && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > $O/c5_new.json 2> $O/c5_new.log && \
CCAMD_LIB=$B timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > $O/c5_base.json 2> $O/c5_base.log && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
