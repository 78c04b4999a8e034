set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_handoff.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -30 $O/pytest.log
exit $rc
