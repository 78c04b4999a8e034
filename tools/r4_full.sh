# full GPU suite + smoke + default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4full
mkdir -p $O
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; p=r['placement']
print(d['value'], d['ms_per_step'], r['frac'], r.get('candidate0_ms'), r.get('kept_ms'), p['candidates_ms'], round(p['peak_device_bytes']/1e9,2))"
