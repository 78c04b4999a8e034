# round-4 profiles after the 2x2x2 pair kernel: C4 trace + PMC, and the
# XY-transposed C2 / C4 bench lines against their live probes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NO_SQ=1 bash tools/profile.sh c4 r04b || exit 1
mkdir -p gpurun_out/r4xy
for c in c2 c4; do
  timeout -k 10 300 python3 bench.py --config $c --xy --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/r4xy/$c.json 2> gpurun_out/r4xy/$c.err || { tail gpurun_out/r4xy/$c.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --config c4 --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/r4xy/c4_plain.json 2> gpurun_out/r4xy/c4p.err || { tail gpurun_out/r4xy/c4p.err; exit 1; }
for f in gpurun_out/r4xy/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$f', r['kernel'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'), r.get('candidate0_ms'))"; done
