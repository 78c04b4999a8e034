set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "3d or c4 or xy" > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,2,512 --instances 3 > $O/c4_ab.txt 2>&1 || { tail $O/c4_ab.txt; exit 1; }
cat $O/c4_ab.txt
timeout -k 10 300 python3 bench.py --config c4 --xy --steps 100 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > $O/c4xy.json 2> $O/c4xy.err || { tail $O/c4xy.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4xy.json')); r=d['roofline']; print('c4 xy', r['kernel'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'))"
