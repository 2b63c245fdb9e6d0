set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c5trace
mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/c5prof.json 2> $R/$O/c5prof.log
