# dev: kernel traces of the e2e codec runs (zstd L1, blosc-zstd bitshuffle)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/trace_e2e.sh zstd1 --e2e pinned --codec zstd || exit 1
bash tools/trace_e2e.sh bzsh2 --e2e pinned --codec blosc-zstd --compress 2 || exit 2
for n in zstd1 bzsh2; do
  f=$(find gpurun_out/trace_e2e/$n -name 'run_kernel_trace.csv' | head -1)
  python3 tools/e2e_kernels.py $f > gpurun_out/trace_e2e/${n}_summary.txt
  echo "== $n"; cat gpurun_out/trace_e2e/${n}_summary.txt
done
