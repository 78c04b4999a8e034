# placement search strategies, fresh process each, twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
rm -f $O/runs.jsonl
run() { timeout -k 10 240 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line --no-hbm-probe "$@" > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/tmp.json')); r=d['roofline']; p=r['placement']; print(json.dumps({'args': sys.argv[1:], 'frac': r['frac'], 'ms': r['kernel_avg_ms'], 'c0': r.get('candidate0_ms'), 'kept': p['kept'], 'n': len(p['candidates_ms']), 'peak_gb': round(p['peak_device_bytes']/1e9,2)}))" "$@" >> $O/runs.jsonl; }
for rep in 1 2; do
run --placement-tries 16
run --placement-tries 16 --tune placement_spacer_bytes=2147483648
run --placement-tries 16 --tune placement_spacer_bytes=4294967296 --tune ring_malloc_flags=4
run --placement-tries 16 --tune placement_spacer_bytes=4294967296
run --placement-tries 12 --tune placement_mode=1 --tune ring_malloc_flags=4
done
cat $O/runs.jsonl
