# End-to-end sweep of one box: raw / lz4 / zstd hand-offs (bench.py --e2e),
# the paced C3 camera and the shard-file example.  One JSON line per run in
# gpurun_out/${TAG}_e2e.jsonl and gpurun_out/${TAG}_fs_e2e.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02}
OUT=gpurun_out/${TAG}_e2e.jsonl
FS=gpurun_out/${TAG}_fs_e2e.jsonl
: > $OUT
: > $FS
run() {
    timeout -k 10 240 python3 bench.py --steps 16 --warmup 2 "$@" \
        > gpurun_out/e2e_tmp.log 2>&1 || { tail -20 gpurun_out/e2e_tmp.log; return 1; }
    grep '^{' gpurun_out/e2e_tmp.log | tail -1 >> $OUT
    tail -1 $OUT | cut -c1-220
}
fs() {
    rm -rf /tmp/aqz_fs
    timeout -k 10 240 ./acquire-zarr_amd/examples/stream_to_filesystem /tmp/aqz_fs \
        --frames 2048 --ring 128 --writers 16 --pattern camera "$@" \
        > gpurun_out/fs_tmp.log 2>&1 || { tail -20 gpurun_out/fs_tmp.log; return 1; }
    grep '^{' gpurun_out/fs_tmp.log | tail -1 >> $FS
    tail -1 $FS | cut -c1-240
}
run --e2e pinned && run --e2e pageable && run --e2e pinned --compress 1 &&
run --e2e pinned --compress 2 && run --e2e pinned --codec blosc-zstd --compress 1 &&
run --e2e pinned --codec blosc-zstd --compress 2 && run --e2e pinned --codec zstd &&
run --e2e pinned --config c3 --compress 2 &&
run --e2e pinned --config c3 --fps 500 --seconds 5 || exit 1
[ -n "$NO_FS" ] && exit 0
fs --config c2 --codec lz4 --shuffle 2 --no-write && fs --config c2 --codec lz4 --shuffle 1 --no-write &&
fs --config c2 --codec raw --no-write && fs --config c2 --codec lz4 --shuffle 2 &&
fs --config c2 --codec lz4 --shuffle 1 && fs --config c2 --codec raw &&
fs --config c3 --codec lz4 --shuffle 2 && fs --config c2 --codec blosc-zstd --shuffle 2 --frames 512
rm -rf /tmp/aqz_fs
