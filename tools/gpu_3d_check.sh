# 3-D parity (all three 2x2x2 kernels) + same-stage C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "3d or c4" > gpurun_out/p3d.log 2>&1
rc=$?; tail -3 gpurun_out/p3d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/knob_ab.py --config c4 --instances 3 --knobs 0,1024,256
