# dev: C4 128- vs 256-plane launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  for b in 128 256; do
    timeout -k 10 180 python3 bench.py --config c4 --batch $b --steps 200 --warmup 10 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/c4_tmp.json 2> gpurun_out/c4_tmp.err || { tail gpurun_out/c4_tmp.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c4_tmp.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c4 batch $b', d['value'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'))"
  done
done
