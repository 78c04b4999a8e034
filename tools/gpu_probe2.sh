set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/pcie_probe.py || exit 1
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-pyramid-only-line | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('events   ', d['ms_per_step'], d['roofline']['kernel_avg_ms'])" || exit 2
timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-pyramid-only-line --no-kernel-events | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('no events', d['ms_per_step'], d['roofline']['kernel_avg_ms'])" || exit 3
done
timeout -k 10 200 python3 bench.py --config c3 --e2e pinned --fps 500 --seconds 5 || exit 4
