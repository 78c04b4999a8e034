# dev: strip kernel with / without the level 0-2 has_data stores (knob 32), pyramid-only and full C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  for k in 0 32; do
    for extra in "--pyramid-only" ""; do
      timeout -k 10 180 python3 bench.py --config c2 --tune knobs=$k $extra --steps 400 --warmup 10 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/fl_tmp.json 2> gpurun_out/fl_tmp.err || { tail gpurun_out/fl_tmp.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/fl_tmp.json').read().strip().splitlines()[-1]); r=d['roofline']; print('knobs=$k $extra', r['kernel_avg_ms'], round(r['achieved'],1), 'kept', r['placement'].get('kept_ms_final'))"
    done
  done
done
