set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
rm -f $O/sweep.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_handoff.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "replay or slab" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for args in "--copy-threads 8 --host-slots 3" "--copy-threads 8 --batch 128" "--copy-threads 6" "--copy-threads 8 --pool-threads 8"; do
  echo "# $args" >> $O/sweep.jsonl
  timeout -k 10 200 python3 -u tools/binding_e2e.py --frames 2048 --codecs raw,lz4,zstd-1 $args >> $O/sweep.jsonl 2> $O/sweep.err || { tail $O/sweep.err; exit 1; }
done
for src in pageable pinned; do for c in none lz4; do
  timeout -k 10 200 python3 bench.py --config c2-ref4 --e2e $src --codec $c --compress 1 --steps 16 --warmup 2 >> $O/bench_e2e.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
done; done
cat $O/sweep.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('#'): print(l.strip()); continue
    d=json.loads(l); print(d['codec_name'], d['input_gbs'], d['seconds'])"
python3 -c "
import json
for l in open('$O/bench_e2e.jsonl'):
    d=json.loads(l); print(d['config']['workload'][-30:], d['metric'][-60:], d['value'])"
