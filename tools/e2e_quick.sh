# dev: e2e codec rows (pinned source)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/e2e_quick.jsonl
for a in "$@"; do
  timeout -k 10 240 python3 bench.py --steps 16 --warmup 2 --e2e pinned $a > gpurun_out/e2e_tmp.log 2>&1 || { tail -20 gpurun_out/e2e_tmp.log; exit 2; }
  grep '^{' gpurun_out/e2e_tmp.log | tail -1 >> gpurun_out/e2e_quick.jsonl
  grep '^{' gpurun_out/e2e_tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'], d.get('d2h_gbs_per_gpu'), d.get('sink_bytes_per_input_byte'), d['config'].get('clevel'))"
done
