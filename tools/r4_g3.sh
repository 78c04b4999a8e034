# placement: contiguous ring allocations vs default, fresh process per run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
for i in 1 2 3; do
for fl in 4 0; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --ring-flags $fl --plan "start,all,all,all,all" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
done
cat $O/plans.jsonl
