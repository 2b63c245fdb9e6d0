set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fin
R=$(pwd)
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/fin/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/fin/c2_bench.json 2> gpurun_out/fin/c2_bench.log && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/c2prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/fin/c2prof_bench.json 2> $R/gpurun_out/fin/c2prof_bench.log && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/fin/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/fin/pmc_fetch.json 2> $R/gpurun_out/fin/pmc_fetch.log && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/fin/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/fin/pmc_write.json 2> $R/gpurun_out/fin/pmc_write.log && \
cd $R && python3 scripts/pmc_traffic.py gpurun_out/fin/pmc_fetch/run_counter_collection.csv gpurun_out/fin/pmc_write/run_counter_collection.csv gpurun_out/fin/pmc_c2_traffic.json 3 gpurun_out/fin/pmc_fetch.json
