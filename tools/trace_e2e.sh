# rocprofv3 kernel + memory-copy trace of an end-to-end bench run
#   tools/trace_e2e.sh NAME [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NAME=${1:-pinned}; shift
OUT=gpurun_out/trace_e2e
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/$NAME -o run -- python3 bench.py --config c2 --steps 8 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench_$NAME.log 2>&1 || exit 1
