# rocprofv3 kernel trace + PMC passes of the default bench (one command per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${1:-c2}
TAG=${2:-r01}
OUT=gpurun_out/prof_${TAG}_${CFG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit 1
tail -1 $OUT/bench_trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_write.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_sq.log 2>&1 || exit 4
find $OUT -name "*.csv" | head -20
