# SQ counter passes over the codec bench (one payload): instruction mix and
# LDS stalls of lz4_streams.   tools/pmc_codec.sh TAG [codec_bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_codec_${1:-x}
mkdir -p $OUT
A="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
B="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL"
timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d $OUT/a -o run -- python3 tools/codec_bench.py --reps 1 ${@:2} > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $B --output-format csv -d $OUT/b -o run -- python3 tools/codec_bench.py --reps 1 ${@:2} > $OUT/b.log 2>&1 || exit 2
