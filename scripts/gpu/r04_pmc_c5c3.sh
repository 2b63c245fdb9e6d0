set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc53
mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
cd /tmp && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$O/c5_fetch -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/$O/c5_fetch.json 2> $R/$O/c5_fetch.log && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$O/c5_write -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/$O/c5_write.json 2> $R/$O/c5_write.log && \
cd $R && python3 scripts/pmc_traffic.py $O/c5_fetch/run_counter_collection.csv $O/c5_write/run_counter_collection.csv $O/pmc_c5_traffic.json 3 $O/c5_fetch.json > /dev/null && \
cd /tmp && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/$O/c3_fetch -o run --output-format csv -- python3 $R/bench.py --config c3 --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/$O/c3_fetch.json 2> $R/$O/c3_fetch.log && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/$O/c3_write -o run --output-format csv -- python3 $R/bench.py --config c3 --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/$O/c3_write.json 2> $R/$O/c3_write.log && \
cd $R && python3 scripts/pmc_traffic.py $O/c3_fetch/run_counter_collection.csv $O/c3_write/run_counter_collection.csv $O/pmc_c3_traffic.json 3 $O/c3_fetch.json > /dev/null
