# round 3 (dev): headline test at the 256-frame C2 launch, its profiles, the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_headline.py -m gpu -q -x --timeout 500 --timeout-method thread -p no:cacheprovider -k "c2" > gpurun_out/headline.log 2>&1 || { tail -30 gpurun_out/headline.log; exit 1; }
tail -2 gpurun_out/headline.log
bash tools/profile.sh c2 r03b || exit 2
bash tools/profile.sh c2 r03b pyr || exit 3
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 4
cat gpurun_out/bench_default.json
