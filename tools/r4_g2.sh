# placement localisation, one process per plan (fresh allocator state each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
for plan in "start,src,src" "start,L=0x1e" "start,L=0x2,L=0x4,L=0x8,L=0x10" \
            "start,L=0x10,L=0x8,L=0x4,L=0x2" "pre=4096,start" "pre=16384,start" \
            "start,L=1,L=1,L=1" "start,all,all" "start,src,L=0x1e,L=1"; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --plan "$plan" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
cat $O/plans.jsonl
