set -o pipefail
cd $GRAFT_REPO_ROOT
echo "host: $(nproc) cpus; $(rocm-smi --showproductname 2>/dev/null | grep -m1 -i 'card series' || true)"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/bench1.log 2>&1; rc=$?; cat gpurun_out/bench1.log | tail -5; exit $rc
