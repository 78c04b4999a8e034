# XCD walk rotation / frame skew vs placement bands (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rot2
mkdir -p $O
timeout -k 10 300 python3 -u tools/rot_probe.py --knobs 0,2048,524288,526336 --stages 10 --rounds 3 > $O/c2.txt 2>&1 || exit 1
cat $O/c2.txt
timeout -k 10 300 python3 -u tools/rot_probe.py --config c4 --knobs 0,2048 --stages 8 --rounds 3 > $O/c4.txt 2>&1 || exit 2
cat $O/c4.txt
