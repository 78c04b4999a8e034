# round 3: bench line of every BASELINE configuration (one box), plus C3 / C5 at 2x launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03_bench_all.jsonl
mkdir -p gpurun_out
: > $OUT
for a in "--config c2" "--config c2-ref4" "--config c3" "--config c3 --batch 64" "--config c4" "--config c5" "--config c5 --batch 8" "--config c2 --xy"; do
  timeout -k 10 300 python3 bench.py $a --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/ba.log 2>&1 || { tail -5 gpurun_out/ba.log; exit 1; }
  grep '^{' gpurun_out/ba.log | tail -1 >> $OUT
  tail -1 $OUT | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$a', d['value'], 'GB/s in;', r['achieved'], 'GB/s alg; frac', r['frac'], '; of probe', r.get('frac_of_probed_ceiling'), ';', r['kernel'], r['kernel_avg_ms'], 'ms', d.get('pyramid_only', {}).get('kernel_input_frac_of_probed_ceiling'))"
done
