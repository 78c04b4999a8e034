# round-4 profiles: rocprofv3 trace + PMC of the headline (and pyramid-only),
# then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NO_SQ=1 bash tools/profile.sh c2 r04 || exit 1
NO_SQ=1 bash tools/profile.sh c2 r04 pyr || exit 1
NO_SQ=1 bash tools/profile.sh c4 r04 || exit 1
mkdir -p gpurun_out/r4bench
timeout -k 10 600 python3 bench.py > gpurun_out/r4bench/bench_default.json 2> gpurun_out/r4bench/bench_default.err || { tail gpurun_out/r4bench/bench_default.err; exit 1; }
cat gpurun_out/r4bench/bench_default.json
