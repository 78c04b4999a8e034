# End-to-end sweep of one box: raw / lz4 / zstd hand-offs, pinned source,
# C2 frames.  One JSON line per run in gpurun_out/${TAG}_e2e.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02}
OUT=gpurun_out/${TAG}_e2e.jsonl
: > $OUT
run() {
    timeout -k 10 240 python3 bench.py --e2e pinned --steps 16 --warmup 2 "$@" \
        > gpurun_out/e2e_tmp.log 2>&1 || { tail -20 gpurun_out/e2e_tmp.log; return 1; }
    grep '^{' gpurun_out/e2e_tmp.log | tail -1 >> $OUT
    tail -1 $OUT | cut -c1-220
}
run && run --compress 1 && run --compress 2 && run --codec blosc-zstd --compress 1 &&
run --codec blosc-zstd --compress 2 && run --codec zstd && run --config c3 --compress 2
