set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
K=0,$((2<<13)),$((3<<13)),$((4<<13)),$((5<<13)),$((6<<13))
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --knobs $K --instances 2 > $O/occ_ab2.txt 2>&1 || { tail $O/occ_ab2.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --knobs $K --instances 2 --placement-tries 16 >> $O/occ_ab2.txt 2>&1 || { tail $O/occ_ab2.txt; exit 1; }
cat $O/occ_ab2.txt
