# rocprofv3 kernel trace of the codec bench (per-kernel times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_codec_${1:-x}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/codec_bench.py --reps 2 ${@:2} > $OUT/bench.log 2>&1 || exit 1
cat $OUT/bench.log | grep -v amdgpu.ids
f=$(find $OUT -name "*kernel_stats.csv" | head -1); cat "$f" | cut -d, -f1-8 | head -12
