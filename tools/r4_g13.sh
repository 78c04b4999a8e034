set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,2,0,2 --instances 3 --placement-tries 16 > $O/c4_ab_search.txt 2>&1 || { tail $O/c4_ab_search.txt; exit 1; }
cat $O/c4_ab_search.txt
