# GPU parity suite without -x (every failure listed), then smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -30
echo "pytest rc=$rc"
exit $rc
