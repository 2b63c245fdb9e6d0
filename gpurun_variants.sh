#!/bin/bash
# bench the default build and each in-tree tuning variant back to back (same input)
mkdir -p gpurun_out
for v in "" ${VARIANTS}; do
  if [ -z "$v" ]; then tag=default; lib=""; else tag=$v; lib=$(pwd)/consensuscruncher_amd/lib/variants/libccamd_$v.so; fi
  CCAMD_LIB=$lib timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/var_$tag.json 2> gpurun_out/var_$tag.log || exit $?
done
