set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/trace_e2e
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/${1:-pinned} -o run -- python3 bench.py --config c2 --e2e ${1:-pinned} --steps 6 --warmup 2 > $OUT/bench_${1:-pinned}.log 2>&1 || exit 1
find $OUT -name "*.csv" | head
