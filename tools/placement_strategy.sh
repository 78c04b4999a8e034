# placement-search strategies (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/strat
mkdir -p $O
timeout -k 10 400 python3 -u tools/placement_strategy.py --rounds 3 > $O/strat.jsonl 2>&1 || exit 1
cat $O/strat.jsonl
