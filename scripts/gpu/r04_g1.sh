set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r04_base_c2_bench.json 2> gpurun_out/r04_base_c2_bench.log && \
timeout -k 10 700 python bench.py --no-cpu-baseline --config c3 --steps 5 --warmup 1 > gpurun_out/r04_c3n1_bench.json 2> gpurun_out/r04_c3n1_bench.log
