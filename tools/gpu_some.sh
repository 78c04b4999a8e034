# run selected GPU tests (dev): tools/gpu_some.sh "<pytest -k expr or node ids>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/some
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest $1 -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -25 $O/pytest.log
exit $rc
