#!/usr/bin/env bash
# Kernel + memory-copy timeline of one e2e bench line (rocprofv3, no PMC):
#   gpurun -- bash tools/e2e_trace.sh <tag> <bench args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/e2e_$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline "$@" > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-400
