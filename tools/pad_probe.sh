# placement bands vs chunk pitch stagger, pads interleaved in one process (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pad2
mkdir -p $O
timeout -k 10 300 python3 -u tools/pad_probe.py --interleave --stages 4 --pads 0,16384,270336,1052672,2101248 > $O/pad.txt 2>&1 || exit 1
cat $O/pad.txt
timeout -k 10 300 python3 -u tools/pad_probe.py --interleave --stages 4 --pads 0,1052672,4096,528384 > $O/pad_b.txt 2>&1 || exit 2
cat $O/pad_b.txt
