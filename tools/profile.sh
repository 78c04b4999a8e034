# rocprofv3 kernel trace + PMC passes of one bench configuration (one
# command per pass; PMC never combined with trace domains).
#   tools/profile.sh CFG TAG [pyr]   (pyr: --pyramid-only, named CFG-pyr)
# BENCH_EXTRA: more bench.py arguments (e.g. "--tune knobs=2"), with
# NAME_SUFFIX naming the variant; SQ2: a second SQ pass of these counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${1:-c2}
TAG=${2:-r02}
# trace pass: enough steps that the stage's creation-time placement
# calibration launches (<= 24, same kernel) move the average by < 1%
STEPS=${STEPS:-200}
NAME=$CFG
EXTRA="--no-cpu-baseline --no-pyramid-only-line --no-hbm-probe $BENCH_EXTRA"
if [ "$3" = "pyr" ]; then NAME=$CFG-pyr; EXTRA="$EXTRA --pyramid-only"; fi
NAME=$NAME$NAME_SUFFIX
OUT=gpurun_out/prof_${TAG}_${NAME}
mkdir -p $OUT
echo "python3 bench.py --config $CFG --steps $STEPS --warmup 5 $EXTRA" > $OUT/bench_cmd.txt
sha256sum acquire-zarr_amd/libaqz_gpu.so | cut -d' ' -f1 > $OUT/lib.sha256
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $CFG --steps $STEPS --warmup 5 $EXTRA > $OUT/bench_trace.log 2>&1 || exit 1
tail -1 $OUT/bench_trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 $EXTRA > $OUT/bench_fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 $EXTRA > $OUT/bench_write.log 2>&1 || exit 3
[ -n "$NO_SQ" ] && exit 0
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 $EXTRA > $OUT/bench_sq.log 2>&1 || exit 4
if [ -n "$SQ2" ]; then
timeout -k 10 300 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT/pmc_sq2 -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 $EXTRA > $OUT/bench_sq2.log 2>&1 || exit 5
fi
