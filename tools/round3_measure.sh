# round-3 measurements (dev): read-shape probe; launch-size A/B; XY storage
# order fused vs separate pass; rocprofv3 trace + PMC of C2, C2 pyramid-only
# and C3 (tools/profile.sh, tag r03)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/shape_probe > gpurun_out/shape_probe.txt 2>&1 || { cat gpurun_out/shape_probe.txt; exit 1; }
cat gpurun_out/shape_probe.txt
: > gpurun_out/batch_ab.jsonl
ab() { # $1 = env assignment or "-", $2 = bench args
  if [ "$1" = "-" ]; then
    timeout -k 10 180 python3 bench.py $2 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err || { tail gpurun_out/ab_tmp.err; return 5; }
  else
    env $1 timeout -k 10 180 python3 bench.py $2 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err || { tail gpurun_out/ab_tmp.err; return 5; }
  fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); d['args']='$2'; d['env']='$1'; print(json.dumps(d))" >> gpurun_out/batch_ab.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', '$2', d['value'], r['kernel'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'), r['placement'].get('candidates_ms'))"
}
for a in "--config c3 --batch 32" "--config c3 --batch 64" "--config c2 --pyramid-only --batch 128" "--config c2 --pyramid-only --batch 256"; do
  ab - "$a --steps 400 --warmup 10" || exit 5
done
for i in 1 2; do
  ab - "--config c2 --xy --steps 400 --warmup 10" || exit 6
  ab - "--config c2 --xy --tune knobs=4096 --steps 400 --warmup 10" || exit 6
done
bash tools/profile.sh c2 r03 || exit 2
bash tools/profile.sh c2 r03 pyr || exit 3
bash tools/profile.sh c3 r03 || exit 4
echo done
