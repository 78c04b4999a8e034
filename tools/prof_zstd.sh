# Device zstd kernels in isolation (tools/codec_bench.py) + the GPU zstd tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_zstd.py > gpurun_out/zstd_tests.log 2>&1 || { tail -30 gpurun_out/zstd_tests.log; exit 1; }
tail -2 gpurun_out/zstd_tests.log
for a in "--codec blosc-zstd --shuffle 1" "--codec blosc-zstd --shuffle 2" "--codec zstd --shuffle 0" "--codec lz4 --shuffle 1"; do
  timeout -k 10 200 python3 tools/codec_bench.py --reps 5 $a 2>&1 | grep -v amdgpu.ids || exit 2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zprof2 -o run -- python3 tools/codec_bench.py --reps 5 --codec blosc-zstd --shuffle 1 --kinds camera > gpurun_out/zprof2.log 2>&1 || exit 3
f=$(find gpurun_out/zprof2 -name 'run_kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -12
