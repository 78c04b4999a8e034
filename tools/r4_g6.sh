set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_handoff.py tests/test_gpu_golden.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -40 $O/pytest.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 -u tools/binding_e2e.py > $O/binding_e2e.jsonl 2> $O/binding_e2e.err || { tail $O/binding_e2e.err; exit 1; }
cat $O/binding_e2e.jsonl
