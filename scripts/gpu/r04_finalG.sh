set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/finG
mkdir -p $O
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_bench.json 2> $O/c4_bench.log && \
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > $O/c5_bench.json 2> $O/c5_bench.log && \
timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline --steps 5 > $O/c3_bench.json 2> $O/c3_bench.log && \
CC_BENCH_DEVICES=1 timeout -k 10 600 python bench.py --gpus 2 --no-cpu-baseline --steps 3 --warmup 1 > $O/rehearse2_bench.json 2> $O/rehearse2_bench.log
