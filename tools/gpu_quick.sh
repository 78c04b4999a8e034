# run selected GPU tests (dev): bash tools/gpu_quick.sh "<pytest args>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest $1 -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -30 $O/pytest.log
exit $rc
