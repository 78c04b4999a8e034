# A/B kernel switches on the same stages for every config (tools/ab.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
V=${1:-0:0,64:0,128:0,192:0}
for c in c2 c1 c3 c4 c5; do
timeout -k 10 200 python3 tools/ab.py --config $c --variants $V --stages 2 2>&1 | grep -v amdgpu.ids || exit 1
done
