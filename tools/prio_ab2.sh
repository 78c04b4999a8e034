# e2e stream-priority A/B: copies (AQZ_COPY_PRIORITY) vs compression (AQZ_COMP_PRIORITY)
set -o pipefail
cd $GRAFT_REPO_ROOT
for codec in "--codec blosc-zstd --compress 1" "--codec lz4 --compress 1"; do
  for env in "AQZ_COPY_PRIORITY=1 AQZ_COMP_PRIORITY=0" "AQZ_COPY_PRIORITY=2 AQZ_COMP_PRIORITY=0" "AQZ_COPY_PRIORITY=1 AQZ_COMP_PRIORITY=1" "AQZ_COPY_PRIORITY=0 AQZ_COMP_PRIORITY=1"; do
    env $env timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --e2e pinned $codec > gpurun_out/pa.log 2>&1 || { tail -5 gpurun_out/pa.log; exit 1; }
    echo "$codec | $env | $(grep '^{' gpurun_out/pa.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
