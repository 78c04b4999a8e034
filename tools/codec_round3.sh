# round-3 zstd encoder: codec bench per level/mode, e2e rows, kernel stats (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/codec3
mkdir -p $O
: > $O/codec_bench.txt
for a in "--codec zstd --shuffle 0 --clevel 1" "--codec zstd --shuffle 0 --clevel 3" "--codec zstd --shuffle 0 --clevel 9" \
         "--codec blosc-zstd --shuffle 1 --clevel 5" "--codec blosc-zstd --shuffle 2 --clevel 5" "--codec lz4 --shuffle 1 --clevel 5"; do
  echo "== $a" >> $O/codec_bench.txt
  timeout -k 10 300 python3 tools/codec_bench.py $a --kinds camera,dim,random >> $O/codec_bench.txt 2>&1 || { tail -20 $O/codec_bench.txt; exit 1; }
done
cat $O/codec_bench.txt
: > $O/e2e_zstd.jsonl
for a in "--codec blosc-zstd --compress 1" "--codec blosc-zstd --compress 2" "--codec zstd"; do
  timeout -k 10 240 python3 bench.py --steps 16 --warmup 2 --e2e pinned $a > $O/e2e_tmp.log 2>&1 || { tail -20 $O/e2e_tmp.log; exit 2; }
  grep '^{' $O/e2e_tmp.log | tail -1 >> $O/e2e_zstd.jsonl
  grep '^{' $O/e2e_tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'], d.get('d2h_gbs_per_gpu'), d.get('sink_bytes_per_input_byte'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/zprof -o run -- python3 tools/codec_bench.py --codec zstd --shuffle 0 --clevel 3 --kinds camera,dim --reps 3 > $O/zprof.log 2>&1 || exit 3
f=$(find $O/zprof -name 'run_kernel_stats.csv' | head -1); cp $f $O/zstd_l3_kernel_stats.csv; cut -d, -f1-8 $f | head -20
