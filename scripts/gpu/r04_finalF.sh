set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fin
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fin/c4_bench.json 2> gpurun_out/fin/c4_bench.log && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > gpurun_out/fin/c5_bench.json 2> gpurun_out/fin/c5_bench.log && \
timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline --steps 5 > gpurun_out/fin/c3_bench.json 2> gpurun_out/fin/c3_bench.log
