# GPU parity suite, smoke and a short default bench line (one gpurun call).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "host: $(nproc) cpus"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1; rc=$?; tail -3 gpurun_out/bench1.log; exit $rc
