# Codec kernel profile + end-to-end hand-off measurements (one gpurun call):
#   tools/measure_e2e.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
bash tools/prof_codec.sh ${TAG}_sh1 --reps 5 --shuffle 1 || exit 1
bash tools/prof_codec.sh ${TAG}_sh2 --reps 5 --shuffle 2 || exit 2
E=gpurun_out/e2e_${TAG}.log
: > $E
for args in "--e2e pinned" "--e2e pageable" "--e2e pinned --compress 1" "--e2e pinned --compress 2"; do
  timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline $args >> $E 2>&1 || exit 3
done
timeout -k 10 200 python3 bench.py --config c3 --e2e pinned --fps 500 --seconds 5 >> $E 2>&1 || exit 4
grep '"metric"' $E
