# Same-box A/B of two builds of the library (AQZ_LIB), alternating runs:
#   bash tools/ab_bench.sh CONFIG ROUNDS libA.so libB.so [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=$1; N=$2; A=$3; B=$4; shift 4
for i in $(seq $N); do
  for L in $A $B; do
    AQZ_LIB=$L timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline --no-pyramid-only-line "$@" 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$L', d['value'], r['kernel_avg_ms'], r['frac'], r['placement']['candidates_ms'], r['placement']['kept'])" || exit 1
  done
done
