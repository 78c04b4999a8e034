# parity (incl. the hand-off pipeline test), then end-to-end runs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for src in pinned pageable; do
  timeout -k 10 300 python3 bench.py --config ${1:-c2} --e2e $src --steps ${2:-16} --warmup 2 2>&1 | grep '"metric"' || exit 1
done
timeout -k 10 200 python3 bench.py --config c3 --e2e pinned --fps 500 --seconds 5 2>&1 | grep '"metric"' || exit 2
