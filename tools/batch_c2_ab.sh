# dev: C2 full stage, 128- vs 256-frame launches, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  for b in 128 256; do
    timeout -k 10 180 python3 bench.py --config c2 --batch $b --steps 300 --warmup 10 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/b_tmp.json 2> gpurun_out/b_tmp.err || { tail gpurun_out/b_tmp.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/b_tmp.json').read().strip().splitlines()[-1]); r=d['roofline']; print('batch $b', d['value'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'), 'kept', r['placement'].get('kept_ms_final'), 'n', len(r['placement'].get('candidates_ms', [])))"
  done
done
