# round-3 device zstd: GPU zstd tests, codec bench per level / mode, e2e rows (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/codec3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_fs_sink.py -m gpu -q -x -p no:cacheprovider > $O/zt.log 2>&1 || { tail -30 $O/zt.log; exit 3; }
tail -1 $O/zt.log
: > $O/codec_bench.txt
for a in "--codec zstd --shuffle 0 --clevel 1" "--codec zstd --shuffle 0 --clevel 3" "--codec zstd --shuffle 0 --clevel 9" \
         "--codec blosc-zstd --shuffle 1 --clevel 5" "--codec blosc-zstd --shuffle 2 --clevel 1" "--codec blosc-zstd --shuffle 2 --clevel 5" \
         "--codec lz4 --shuffle 1 --clevel 5" "--codec lz4 --shuffle 2 --clevel 5"; do
  echo "== $a" >> $O/codec_bench.txt
  timeout -k 10 300 python3 tools/codec_bench.py $a --kinds camera,dim,random 2>&1 | grep -v amdgpu.ids >> $O/codec_bench.txt || { tail -20 $O/codec_bench.txt; exit 1; }
done
cat $O/codec_bench.txt
: > $O/e2e_zstd.jsonl
for a in "--codec blosc-zstd --compress 1" "--codec blosc-zstd --compress 2" "--codec zstd" "--codec zstd --clevel 3" "--codec lz4 --compress 2"; do
  timeout -k 10 240 python3 bench.py --steps 16 --warmup 2 --e2e pinned $a > $O/e2e_tmp.log 2>&1 || { tail -20 $O/e2e_tmp.log; exit 2; }
  grep '^{' $O/e2e_tmp.log | tail -1 >> $O/e2e_zstd.jsonl
  grep '^{' $O/e2e_tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'], d.get('d2h_gbs_per_gpu'), d.get('sink_bytes_per_input_byte'), d['config'].get('clevel'))"
done
