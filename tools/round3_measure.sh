# round-3 measurements (dev): read-shape probe, then rocprofv3 trace + PMC
# of C2, C2 pyramid-only and C3 (tools/profile.sh, tag r03)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/shape_probe > gpurun_out/shape_probe.txt 2>&1 || { cat gpurun_out/shape_probe.txt; exit 1; }
cat gpurun_out/shape_probe.txt
# launch-tail A/B: frames per launch (each line has its own live probe)
: > gpurun_out/batch_ab.jsonl
for a in "--config c3 --batch 32" "--config c3 --batch 64" "--config c2 --pyramid-only --batch 128" "--config c2 --pyramid-only --batch 256" \
         "--config c3 --batch 32" "--config c3 --batch 64" "--config c2 --pyramid-only --batch 128" "--config c2 --pyramid-only --batch 256"; do
  timeout -k 10 180 python3 bench.py $a --steps 400 --warmup 10 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err || { tail gpurun_out/ab_tmp.err; exit 5; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); d['args']='$a'; print(json.dumps(d))" >> gpurun_out/batch_ab.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$a', r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'), r['placement']['candidates_ms'])"
done
bash tools/profile.sh c2 r03 || exit 2
bash tools/profile.sh c2 r03 pyr || exit 3
bash tools/profile.sh c3 r03 || exit 4
echo done
