#!/bin/bash
# Full-size bench (default args), a rocprofv3 kernel-trace/stats pass, then (PMC=1) the HBM byte
# counters of every kernel: FETCH_SIZE and WRITE_SIZE in separate runs (MI355X_MICROARCH.md,
# rocprofv3 section).  The PMC runs make 3 pipeline passes (setup + 1 profiling + 1 timed step).
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.log || exit $?
if [ -n "$PMC" ]; then
  timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/pmc_fetch.json 2> $R/gpurun_out/pmc_fetch.log || exit $?
  timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/pmc_write.json 2> $R/gpurun_out/pmc_write.log || exit $?
  cd $R && python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv gpurun_out/pmc_traffic.json 3 gpurun_out/pmc_fetch.json
fi
