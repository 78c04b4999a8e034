# HISTORICAL (rounds 2-3): the environment switch this script sets was removed in
# round 4 (tuning is only in aqz_stage_bench_options); kept for the provenance of
# the profiles/ files it produced.
# A/B of the PCIe stream priority (AQZ_COPY_PRIORITY) on the e2e path.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prio_ab.txt
: > $OUT
one() {
    local tag="$1"; shift
    env "$@" timeout -k 10 200 python3 bench.py --e2e pinned --steps 16 --warmup 2 $ARGS > gpurun_out/prio_tmp.log 2>&1 || { tail -5 gpurun_out/prio_tmp.log; return 1; }
    echo "$tag $ARGS $(grep -o '"value": [0-9.]*' gpurun_out/prio_tmp.log | tail -1)" | tee -a $OUT
}
for ARGS in "--compress 1" "--compress 1"; do
  one high AQZ_COPY_PRIORITY=1 && one normal AQZ_COPY_PRIORITY=0 && one low AQZ_COPY_PRIORITY=2 || exit 1
done
