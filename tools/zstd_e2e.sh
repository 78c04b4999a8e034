set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in "--codec blosc-zstd --compress 1" "--codec blosc-zstd --compress 2" "--codec zstd"; do
  timeout -k 10 200 python3 bench.py --e2e pinned --steps 16 --warmup 2 $a > gpurun_out/ze.log 2>&1 || { tail -20 gpurun_out/ze.log; exit 1; }
  grep '^{' gpurun_out/ze.log | tail -1 | cut -c 90-420
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zprof -o run -- python3 bench.py --e2e pinned --steps 8 --warmup 2 --codec blosc-zstd --compress 1 > gpurun_out/zprof.log 2>&1 || exit 2
f=$(find gpurun_out/zprof -name 'run_kernel_stats.csv' | head -1); cut -d, -f1-8 $f | head -20
