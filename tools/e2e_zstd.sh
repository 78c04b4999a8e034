# e2e rows of the device zstd codecs only (bench.py --e2e pinned)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/${TAG:-r02}_e2e_zstd.jsonl
for a in "--codec blosc-zstd --compress 1" "--codec blosc-zstd --compress 2" "--codec zstd"; do
  timeout -k 10 240 python3 bench.py --steps 16 --warmup 2 --e2e pinned $a > gpurun_out/e2e_tmp.log 2>&1 || { tail -20 gpurun_out/e2e_tmp.log; exit 1; }
  grep '^{' gpurun_out/e2e_tmp.log | tail -1 >> gpurun_out/${TAG:-r02}_e2e_zstd.jsonl
  grep '^{' gpurun_out/e2e_tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'], d.get('d2h_gbs_per_gpu'))"
done
