set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/place2
mkdir -p $O
timeout -k 10 120 tools/region_probe 12 2048 2 > $O/region.txt 2>&1 || exit 1
cat $O/region.txt
for b in 0 16 48; do
  timeout -k 10 120 python3 tools/placement_pmc.py --stages 4 --rounds 2 --reps 10 --ballast-gib $b > $O/ballast$b.txt 2>&1 || exit 2
  echo "ballast $b"; cat $O/ballast$b.txt
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_handoff.py tests/test_gpu_golden.py -q --timeout 120 --timeout-method thread > $O/handoff.txt 2>&1; echo pytest rc=$?; tail -5 $O/handoff.txt
