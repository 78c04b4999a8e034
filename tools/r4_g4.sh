# placement: contiguous rings after a contiguous spacer of S GiB (freed after)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
for S in 0 4 7 9 10.5 12 16 24 48 96 160; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --ring-flags 4 --spacer-gib $S --plan "start,all" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
for S in 12 48; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --ring-flags 0 --spacer-gib $S --plan "start,all" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
cat $O/plans.jsonl
