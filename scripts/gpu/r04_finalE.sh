set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fin
R=$(pwd)
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fin/c4_bench.json 2> gpurun_out/fin/c4_bench.log && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/c4prof -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/fin/c4prof_bench.json 2> $R/gpurun_out/fin/c4prof_bench.log && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/fin/pmc_c4_fetch -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/fin/pmc_c4_fetch.json 2> $R/gpurun_out/fin/pmc_c4_fetch.log && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/fin/pmc_c4_write -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/fin/pmc_c4_write.json 2> $R/gpurun_out/fin/pmc_c4_write.log && \
cd $R && python3 scripts/pmc_traffic.py gpurun_out/fin/pmc_c4_fetch/run_counter_collection.csv gpurun_out/fin/pmc_c4_write/run_counter_collection.csv gpurun_out/fin/pmc_c4_traffic.json 3 gpurun_out/fin/pmc_c4_fetch.json > /dev/null && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > gpurun_out/fin/c5_bench.json 2> gpurun_out/fin/c5_bench.log && \
timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline --steps 5 > gpurun_out/fin/c3_bench.json 2> gpurun_out/fin/c3_bench.log
