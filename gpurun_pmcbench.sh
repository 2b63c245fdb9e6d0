#!/bin/bash
# PMC passes first (FETCH_SIZE, WRITE_SIZE, each its own run) over the roofline scope's kernels,
# reduced into profiles/pmc_latest.json, then the default bench that reads it.
mkdir -p gpurun_out
R=$(pwd)
RX="k_rkey|k_scatter_stream|k_pair_coord|k_pair_resid|k_sscs_vote|k_pair_keys|k_fam_mark"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.json 2> $R/gpurun_out/pmc_fetch.log || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_write.json 2> $R/gpurun_out/pmc_write.log || exit $?
cd $R && python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv gpurun_out/pmc_traffic.json || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_latest.json
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log
