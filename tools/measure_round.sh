# the round's measurement artifacts: the default bench line (with the CPU
# baseline), then rocprof trace + PMC for every bench configuration
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
grep '"metric"' gpurun_out/bench_default.log
for c in c2 c3 c4 c5; do bash tools/profile.sh $c $TAG || exit 2; done
bash tools/profile.sh c2 $TAG pyr || exit 3
