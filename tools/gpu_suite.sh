# full GPU suite, then the default bench line (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 2
cat $O/bench.json
