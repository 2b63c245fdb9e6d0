#!/bin/bash
# PMC HBM bytes (FETCH_SIZE, WRITE_SIZE in separate passes) of one config's bench: CFG=c4 etc.
# Writes gpurun_out/pmc_${CFG}_traffic.json (profiles/pmc_${CFG}_latest.json when committed).
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_${CFG}_fetch -o run --output-format csv -- python3 $R/bench.py --config ${CFG} --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/pmc_${CFG}_fetch.json 2> $R/gpurun_out/pmc_${CFG}_fetch.log || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_${CFG}_write -o run --output-format csv -- python3 $R/bench.py --config ${CFG} --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/pmc_${CFG}_write.json 2> $R/gpurun_out/pmc_${CFG}_write.log || exit $?
cd $R && python3 scripts/pmc_traffic.py gpurun_out/pmc_${CFG}_fetch/run_counter_collection.csv gpurun_out/pmc_${CFG}_write/run_counter_collection.csv gpurun_out/pmc_${CFG}_traffic.json 3 gpurun_out/pmc_${CFG}_fetch.json
