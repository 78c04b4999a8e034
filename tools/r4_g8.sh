set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
rm -f $O/*.jsonl
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u tools/binding_e2e.py --frames 4096 --codecs raw,lz4,lz4-bit,blosc-zstd,zstd-1 >> $O/binding.jsonl 2> $O/b.err || { tail $O/b.err; exit 1; }
done
for src in pageable pinned; do
  timeout -k 10 200 python3 bench.py --config c2-ref4 --e2e $src --steps 32 --warmup 2 >> $O/bench_e2e.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  for c in lz4 zstd; do
  timeout -k 10 200 python3 bench.py --config c2-ref4 --e2e $src --codec $c --compress 1 --steps 32 --warmup 2 >> $O/bench_e2e.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/binding.jsonl'):
    d=json.loads(l); print('binding', d['codec_name'], d['input_gbs'])
for l in open('$O/bench_e2e.jsonl'):
    d=json.loads(l); print('bench', d['config']['workload'][-20:], d['metric'][-45:], d['value'])"
