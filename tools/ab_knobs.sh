# Same-box A/B of tuning knobs (bench option knobs) on one build, alternating runs:
#   bash tools/ab_knobs.sh CONFIG ROUNDS KNOBS_A KNOBS_B [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=$1; N=$2; A=$3; B=$4; shift 4
for i in $(seq $N); do
  for K in $A $B; do
    timeout -k 10 120 python bench.py --config $CFG --tune knobs=$K --no-cpu-baseline --no-pyramid-only-line "$@" 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('knobs=$K', d['value'], r['kernel'], r['kernel_avg_ms'], r['frac'])" || exit 1
  done
done
