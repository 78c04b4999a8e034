set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c2 c2-ref4 c3 c5 c4; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline 2>&1 | grep '"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], 'GB/s in;', d['roofline']['achieved'], 'GB/s alg;', d['roofline']['kernel'], d['roofline']['kernel_avg_ms'], 'ms/launch', d['ms_per_step'], 'ms/step')" || exit 1
done
