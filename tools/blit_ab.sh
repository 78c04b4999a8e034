# e2e: HIP runtime blit settings (PCIe copies as shader blits vs fewer blit workgroups / SDMA)
set -o pipefail
cd $GRAFT_REPO_ROOT
for codec in "--codec blosc-zstd --compress 1" "--codec lz4 --compress 1" "--codec none"; do
  for env in "AQZ_X=0" "DEBUG_CLR_LIMIT_BLIT_WG=16" "DEBUG_CLR_LIMIT_BLIT_WG=64" "GPU_BLIT_ENGINE_TYPE=2"; do
    env $env timeout -k 10 120 python3 bench.py --steps 16 --warmup 2 --e2e pinned $codec > gpurun_out/pa.log 2>&1 || { echo "$codec | $env | failed: $(tail -2 gpurun_out/pa.log | tr '\n' ' ' | cut -c1-200)"; continue; }
    echo "$codec | $env | $(grep '^{' gpurun_out/pa.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["d2h_gbs_per_gpu"])')"
  done
done
