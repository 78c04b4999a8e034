set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/pcie_probe.py || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider -k "handoff or device_resident or baseline" > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
for pm in 8 32 128; do
for src in pinned pageable; do
  AQZ_COPY_PIECE_MB=$pm timeout -k 10 300 python3 bench.py --config c2 --e2e $src --steps 8 --warmup 2 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('piece', $pm, '$src', d['value'], d['h2d_gbs_per_gpu'], d['d2h_gbs_per_gpu'])" || exit 3
done
done
# the multi-rank bench path, rehearsed with 2 ranks sharing this box's GPU (gloo)
AQZ_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --no-pyramid-only-line 2>&1 | grep '"metric"' || exit 4
