# dev: pyramid-only nt-policy A/B (same box, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/nt_ab.txt
for i in 1 2; do
  for nt in 7 3 1 5; do
    timeout -k 10 180 python3 bench.py --config c2 --pyramid-only --tune nt=$nt --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/nt_tmp.json 2> gpurun_out/nt_tmp.err || { tail gpurun_out/nt_tmp.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/nt_tmp.json').read().strip().splitlines()[-1]); r=d['roofline']; p=d['hbm_probe']; print('nt=$nt', r['kernel_avg_ms'], round(r['achieved'],1), 'read3_in', p['read_third_input_gbs'], 'in/probe', round(d['value']/p['read_third_input_gbs'],4), 'cands', r['placement'].get('candidates_ms'))" | tee -a gpurun_out/nt_ab.txt
  done
done
