set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base big4 big8; do
  if [ $v = base ]; then L=""; else L=build/var/$v/libccamd.so; fi
  CCAMD_LIB=$L timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 5 --profile-steps 1 > gpurun_out/r04_g19_c4_$v.json 2> gpurun_out/r04_g19_c4_$v.log || exit $?
done
for v in base sv4; do
  if [ $v = base ]; then L=""; else L=build/var/$v/libccamd.so; fi
  CCAMD_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --profile-steps 1 > gpurun_out/r04_g19_c2_$v.json 2> gpurun_out/r04_g19_c2_$v.log || exit $?
done
