# HISTORICAL (rounds 2-3): the environment switch this script sets was removed in
# round 4 (tuning is only in aqz_stage_bench_options); kept for the provenance of
# the profiles/ files it produced.
# dev: zstd L3 parse cost split (AQZ_ZSTD_DBG: 1 no far verification, 2 no far reads)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pab
mkdir -p $O
for dbg in ${DBGS:-0 1 2}; do
  AQZ_ZSTD_DBG_INVALID=1 AQZ_ZSTD_DBG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$dbg -o run -- python3 tools/codec_bench.py --codec zstd --shuffle 0 --clevel 3 --kinds camera --reps 2 > $O/d$dbg.log 2>&1 || exit 1
  f=$(find $O/d$dbg -name 'run_kernel_stats.csv' | head -1)
  echo "== dbg $dbg"; grep device $O/d$dbg.log || true
  python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'aqz' in r['Name']:
        print(f"  {r['Name'][:50]:50s} avg_ms {float(r['AverageNs'])/1e6:8.3f}")
PY
done
