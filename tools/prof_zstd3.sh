# dev: kernel stats of the device zstd at given settings: tools/prof_zstd3.sh "<codec_bench args>" tag
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zprof3
mkdir -p $O
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr -c 'a-z0-9' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 tools/codec_bench.py $cfg --kinds camera --reps 2 > $O/$tag.log 2>&1 || exit 1
  f=$(find $O/$tag -name 'run_kernel_stats.csv' | head -1); cp $f $O/${tag}_kernel_stats.csv
  echo "== $cfg"; grep -E 'device' $O/$tag.log
  python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'aqz' in r['Name']:
        print(f"  {r['Name'][:64]:64s} n {r['Calls']:>3} avg_ms {float(r['AverageNs'])/1e6:8.3f}")
PY
done
