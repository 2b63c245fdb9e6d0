set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sortfam
mkdir -p $O
R=$(pwd)
B=build/var/base/libccamd.so
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deep_rank.py > $O/deep_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_new1.json 2> $O/c4_new1.log && \
CCAMD_LIB=$B timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_base1.json 2> $O/c4_base1.log && \
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_new2.json 2> $O/c4_new2.log && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_w -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/$O/pmc_w.json 2> $R/$O/pmc_w.log
