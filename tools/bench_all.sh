# Device-resident bench line of every BASELINE configuration (one box, one
# call), with the live HBM probe: gpurun_out/${TAG}_bench_all.jsonl
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r02}
OUT=gpurun_out/${TAG}_bench_all.jsonl
mkdir -p gpurun_out
: > $OUT
for c in c2 c2-ref4 c3 c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/ba.log 2>&1 || { tail -5 gpurun_out/ba.log; exit 1; }
  grep '^{' gpurun_out/ba.log | tail -1 >> $OUT
  tail -1 $OUT | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', d['value'], 'GB/s in;', r['achieved'], 'GB/s alg; frac', r['frac'], '; of probe', r.get('frac_of_probed_ceiling'), ';', r['kernel'], r['kernel_avg_ms'], 'ms')"
done
