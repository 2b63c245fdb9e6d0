#!/bin/bash
# Vote tuning: SSCS-stage kernel timings of the in-tree variants on one BAM, then one SQ PMC pass.
mkdir -p gpurun_out
R=$(pwd)
B=/tmp/c2_vote.bam
timeout -k 10 300 python scripts/vote_bench.py --bam $B --pairs ${PAIRS:-3000000} > gpurun_out/vb_default.json 2> gpurun_out/vb_default.log || exit $?
for v in ${VARIANTS}; do
  CCAMD_LIB=$R/consensuscruncher_amd/lib/variants/libccamd_$v.so timeout -k 10 300 python scripts/vote_bench.py --bam $B \
    > gpurun_out/vb_$v.json 2> gpurun_out/vb_$v.log || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1 || true
if [ -n "$SQPMC" ]; then
  timeout -s KILL 180 rocprofv3 --pmc $SQPMC --kernel-include-regex "${PMC_REGEX:-k_sscs_vote_swar}" -d $R/gpurun_out/pmc_sq -o run \
    --output-format csv -- python3 $R/scripts/vote_bench.py --bam $B --steps 1 > $R/gpurun_out/pmc_sq.json 2> $R/gpurun_out/pmc_sq.log || exit $?
fi
