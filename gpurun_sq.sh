#!/bin/bash
# SQ counters (one pass) and FETCH_SIZE (another) for the kernels matching $REGEX on the full bench
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-include-regex "${REGEX}" -d $R/gpurun_out/sq -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/sq.json 2> $R/gpurun_out/sq.log || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "${REGEX}" -d $R/gpurun_out/fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --profile-steps 1 --no-cpu-baseline > $R/gpurun_out/fetch.json 2> $R/gpurun_out/fetch.log || exit $?
