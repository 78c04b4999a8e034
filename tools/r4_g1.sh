set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "environment or 3d_shallow or xy_fused or async_handoff" > gpurun_out/r4a/pytest.log 2>&1 || { tail -30 gpurun_out/r4a/pytest.log; exit 1; }
tail -3 gpurun_out/r4a/pytest.log
timeout -k 10 300 python3 -u tools/placement_localize.py --trials 5 > gpurun_out/r4a/localize.jsonl 2> gpurun_out/r4a/localize.err || { tail gpurun_out/r4a/localize.err; exit 1; }
tail -2 gpurun_out/r4a/localize.jsonl
