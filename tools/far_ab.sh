# dev: device zstd levels (codec bench, 8 MiB chunks) and the ratio tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/far_ab.txt
for a in "--codec zstd --shuffle 0 --clevel 1" "--codec zstd --shuffle 0 --clevel 3" "--codec zstd --shuffle 0 --clevel 9" "--codec blosc-zstd --shuffle 2 --clevel 5" "--codec blosc-zstd --shuffle 1 --clevel 5"; do
  echo "== $a" >> gpurun_out/far_ab.txt
  timeout -k 10 300 python3 tools/codec_bench.py $a --kinds camera,dim --reps 3 2>&1 | grep -v amdgpu.ids >> gpurun_out/far_ab.txt || { tail -20 gpurun_out/far_ab.txt; exit 1; }
done
cat gpurun_out/far_ab.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_fs_sink.py -m gpu -q -rA -p no:cacheprovider > gpurun_out/zt.log 2>&1; rc=$?
grep -E 'codec [23] shuffle|bytes by|passed|failed|Error' gpurun_out/zt.log | head -40
exit $rc
