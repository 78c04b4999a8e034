# bench every config, then rocprof trace + PMC passes of c2 and c2-ref4
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/bench_all.sh || exit 1
bash tools/profile.sh c2 ${1:-r01} || exit 2
bash tools/profile.sh c2-ref4 ${1:-r01} || exit 3
