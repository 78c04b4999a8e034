set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/zdbg
T='tests/test_gpu_zstd.py -m gpu -k test_stage_blosc_zstd_layers'
for cfg in "0 1" "28672 0" "0 0" "12288 1" "28672 1"; do
  set -- $cfg
  AQZ_ZSTD_HIST=$1 AQZ_ZSTD_FIT=$2 timeout -k 10 300 python3 -m pytest $T -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/zdbg/h$1_f$2.log 2>&1
  echo "hist $1 fit $2: $(tail -1 gpurun_out/zdbg/h$1_f$2.log)"
done
