#!/usr/bin/env bash
# Round-6 GPU runs, one function per gpurun call (the profiles/r06_* files
# come from these):  gpurun -- bash tools/r06_gpu.sh <step> [args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp

# the whole GPU suite + smoke
step_full() {
O=gpurun_out/r6full
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
cat $O/smoke.log
}

# some GPU test files (names after the step)
step_tests() {
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest "$@" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -25 $O/pytest.log
[ $rc -eq 0 ] || exit 1
}

# the default bench line
step_default() {
O=gpurun_out/r6default${1:-}
mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
}

# rocprof trace + PMC of one bench configuration (tools/profile.sh CFG TAG [pyr])
step_prof() {
STEPS=${STEPS:-200} bash tools/profile.sh "$@" || exit 1
}

# start of round: suite + smoke, default line, C2 pyramid-only profile
step_base() {
step_full || exit 1
step_default || exit 1
NO_SQ=${NO_SQ:-} STEPS=200 bash tools/profile.sh c2 r06 pyr || exit 1
}

# pyramid-only: occupancy cap x nontemporal policy on one stage; the
# pyramid-only bench line with its same-memory read-third probe
step_p1() {
O=gpurun_out/r6p1
mkdir -p $O
timeout -k 10 400 python3 -u tools/knob_ab.py --config c2 --pyramid-only --knobs 0,8192,32768,40960,57344 --nts 7,1,0 --instances 2 > $O/pyr_ab.txt 2>&1 || { tail $O/pyr_ab.txt; exit 1; }
cat $O/pyr_ab.txt
for i in 1 2; do
timeout -k 10 200 python3 -u bench.py --pyramid-only --steps 50 --warmup 5 --no-cpu-baseline --no-hbm-probe > $O/pyr$i.json 2> $O/pyr$i.err || { tail $O/pyr$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/pyr$i.json')); r=d['roofline']; p=r['placement']; print(json.dumps({'frac': r['frac'], 'ms': r['kernel_avg_ms'], 'cand': p['candidates_ms'], 'kept': p['kept'], 'exp': p['expected_ms'], 'probe': p['probe_bus_gbs'], 'stop': p.get('stop'), 'fop': r.get('frac_of_probe_same_shape')}))"
done
}

# host split of level 0: parity tests, then the e2e A/B (bench.py --e2e
# pinned / pageable, host vs device level 0; the binding's raw row both ways)
step_p2() {
O=gpurun_out/r6p2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_hostsplit.py tests/test_gpu_handoff.py tests/test_gpu_zstd.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
e2e_ab $O
}

e2e_ab() {
O=$1
for a in "--e2e pinned" "--e2e pinned --level0-split device" "--e2e pageable" "--e2e pageable --level0-split device"; do
timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('$a', d['value'], d['ms_per_step'], d.get('d2h_bytes_per_input_byte'), d.get('level0_split'))"
done
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs raw > $O/binding.jsonl 2> $O/binding.err || { tail $O/binding.err; exit 1; }
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs raw --level0 device >> $O/binding.jsonl 2>> $O/binding.err || { tail $O/binding.err; exit 1; }
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs raw --copy-threads 15 >> $O/binding.jsonl 2>> $O/binding.err || { tail $O/binding.err; exit 1; }
python3 -c "
import json
for l in open('$O/binding.jsonl'):
    d = json.loads(l); print('binding', d['codec_name'], d['level0_split'], d['copy_threads'], d['input_gbs'])"
}

# host split throughput on the box's cores (tools/split_probe.cpp, CPU only)
step_p3() {
O=gpurun_out/r6p3
mkdir -p $O
g++ -O3 -std=c++20 -pthread -DWITH_HIP -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/split_probe.cpp -o $O/split_probe -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib || exit 1
timeout -k 10 300 $O/split_probe 256 > $O/split_probe.jsonl 2>&1 || { tail $O/split_probe.jsonl; exit 1; }
timeout -k 10 300 $O/split_probe 256 pinned >> $O/split_probe.jsonl 2>&1 || { tail $O/split_probe.jsonl; exit 1; }
timeout -k 10 300 $O/split_probe 256 pinned-thp >> $O/split_probe.jsonl 2>&1 || { tail $O/split_probe.jsonl; exit 1; }
grep -i -E "AnonHugePages|Hugepagesize" /proc/meminfo; cat /sys/kernel/mm/transparent_hugepage/enabled || true
cat $O/split_probe.jsonl
nproc; grep -m1 "model name" /proc/cpuinfo; taskset -p $$ || true
}

# host split A/B on one box: streaming vs plain stores (AQZ_SPLIT_NT), split
# threads (AQZ_SPLIT_THREADS) for bench.py --e2e, copy threads for the binding
step_p4() {
O=gpurun_out/r6p4
mkdir -p $O
for nt in 1 0 1 0; do
for a in "--e2e pinned" "--e2e pageable"; do
AQZ_SPLIT_NT=$nt timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('nt=$nt $a', d['value'])"
done
done
for th in 7 11; do
AQZ_SPLIT_THREADS=$th timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 --e2e pinned --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('split threads $th+1 pinned', d['value'])"
done
for nt in 1 0; do
for ct in 8 15; do
AQZ_SPLIT_NT=$nt timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs raw --copy-threads $ct > $O/b.json 2>> $O/binding.err || { tail $O/binding.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); print('binding nt=$nt copy $ct', d['input_gbs'])"
done
done
}

# e2e rows, 3 interleaved rounds on one box (medians for DESIGN): bench.py
# --e2e pinned / pageable with level 0 on the host and on the device, the
# binding's raw row both ways
step_p5() {
O=gpurun_out/r6p5
mkdir -p $O
for rnd in 1 2 3; do
for a in "--e2e pinned" "--e2e pinned --level0-split device" "--e2e pageable" "--e2e pageable --level0-split device"; do
timeout -k 10 200 python3 -u bench.py --steps 48 --warmup 4 $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('r$rnd $a', d['value'], d.get('level0_split'))"
done
for l0 in host device; do
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs raw --level0 $l0 >> $O/binding.jsonl 2>> $O/binding.err || { tail $O/binding.err; exit 1; }
python3 -c "import json; d=[json.loads(l) for l in open('$O/binding.jsonl')][-1]; print('r$rnd binding raw', d['level0_split'], d['input_gbs'])"
done
done
}

# pinned e2e with the host split: split before the append, producer thread
# on the device's NUMA node (A/B, interleaved)
step_p6() {
O=gpurun_out/r6p6
mkdir -p $O
for rnd in 1 2; do
for a in "" "--split-first" "--e2e-numa" "--e2e-numa --split-first"; do
timeout -k 10 200 python3 -u bench.py --steps 48 --warmup 4 --e2e pinned $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('r$rnd pinned $a', d['value'], d['host_threads'])"
done
timeout -k 10 200 python3 -u bench.py --steps 48 --warmup 4 --e2e pageable --e2e-numa --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('r$rnd pageable numa', d['value'])"
done
}

# hand-off replays (the shared ArrayLedger checked against Array's rules),
# then the split probe (pageable vs pinned sources)
step_p7() {
O=gpurun_out/r6p7
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_handoff.py tests/test_gpu_hostsplit.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step_p3
}

# binding e2e (every codec) next to bench.py --e2e pinned / pageable of the
# same codecs on one box, with the hand-off's consumer-time breakdown
step_p8() {
O=gpurun_out/r6p8
mkdir -p $O
timeout -k 10 600 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs raw,lz4,lz4-bit,blosc-zstd,zstd-1,zstd-3 > $O/binding.jsonl 2> $O/binding.err || { tail $O/binding.err; exit 1; }
python3 -c "
import json
for l in open('$O/binding.jsonl'):
    d = json.loads(l); print('binding', d['codec_name'], d['level0_split'], d['input_gbs'], d['seconds'], d['consumer_s'])"
for src in pinned pageable; do
for a in "" "--compress 1" "--compress 2" "--codec blosc-zstd --compress 1" "--codec zstd" "--codec zstd --clevel 3"; do
timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 --e2e $src $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('bench $src $a', d['value'], d.get('level0_split'))"
done
done
}

# the binding itself (oracle/_ref/binding_exec) end to end, every codec,
# interleaved with the replay of its hand-off and bench.py --e2e pageable of
# the same codec on one box (profiles/r06_binding_exec_e2e.jsonl)
step_p13() {
O=gpurun_out/r6p13
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_binding_exec.py -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
declare -A BA=([raw]="" [lz4]="--compress 1" [blosc-zstd]="--codec blosc-zstd --compress 1" [zstd-1]="--codec zstd" [zstd-3]="--codec zstd --clevel 3")
for rnd in 1 2; do
for c in raw lz4 blosc-zstd zstd-1 zstd-3; do
for h in exec replay; do
x=""; [ $h = exec ] && x="--exec"
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs $c $x > $O/b.json 2>> $O/binding.err || { tail $O/binding.err; exit 1; }
cat $O/b.json >> $O/binding.jsonl
python3 -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print('r$rnd', d['harness'], d['codec_name'], round(d['input_gbs'], 2))"
done
timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 --e2e pageable ${BA[$c]} --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('r$rnd bench-pageable $c', d['value'])"
done
done
}

# the binding's copy threads (HandoffOptions::copy_threads) for the raw
# hand-off: 8 / 12 / 16, interleaved, with bench.py --e2e pageable beside
step_p14() {
O=gpurun_out/r6p14
mkdir -p $O
for rnd in 1 2 3; do
for ct in 8 12 16; do
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 --codecs raw --copy-threads $ct > $O/b.json 2>> $O/binding.err || { tail $O/binding.err; exit 1; }
cat $O/b.json >> $O/binding.jsonl
python3 -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print('r$rnd copy $ct', round(d['input_gbs'], 2), d['consumer_s'])"
done
timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 --e2e pageable --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('r$rnd bench-pageable raw', d['value'])"
done
}

# SDMA D2H of compressed frames (AQZ_D2H_SDMA=1) vs the blit kernels: codec
# tests under SDMA, then the e2e codec rows interleaved
step_p9() {
O=gpurun_out/r6p9
mkdir -p $O
AQZ_D2H_SDMA=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_handoff.py -m gpu -v -x --timeout 100 --timeout-method thread -p no:cacheprovider -k "codec or compress or lz4 or zstd" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for rnd in 1 2; do
for sd in 0 1; do
for a in "--compress 1" "--codec blosc-zstd --compress 2" "--codec zstd --clevel 3" "--codec zstd"; do
AQZ_D2H_SDMA=$sd timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 --e2e pinned $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('r$rnd sdma=$sd $a', d['value'], d.get('sink_bytes_per_input_byte'))"
done
done
done
}

# bench lines of every config with the current build (device-resident)
step_lines() {
O=gpurun_out/r6lines${1:-}
mkdir -p $O
for c in c2 c3 c4 c5 c1 c2-ref4; do
timeout -k 10 200 python3 -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { tail $O/$c.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; p=r['placement']; py=d.get('pyramid_only') or {}; print(json.dumps({'cfg': '$c', 'value': d['value'], 'frac': r['frac'], 'ms': r['kernel_avg_ms'], 'kernel': r['kernel'], 'cand': p.get('candidates_ms'), 'acc': p.get('accepted'), 'stop': p.get('stop'), 'probe': r.get('probe_same_shape_gbs'), 'fop': r.get('frac_of_probe_same_shape'), 'traffic': r.get('traffic'), 'pyr': py.get('input_rate_frac_of_peak'), 'pyr_fop_same_mem': py.get('kernel_frac_of_probe_same_memory'), 'est_gb': round(p['estimate_device_bytes']/1e9, 2), 'peak_gb': round(p['peak_device_bytes']/1e9, 2)}))" | tee -a $O/lines.jsonl
done
}

# the final library: suite + smoke, the default line, every config's line
step_finala() {
step_full || exit 1
step_default final || exit 1
step_lines final || exit 1
}

# the final library: rocprof trace + PMC of every config (and C2 pyramid-only)
step_finalb() {
for c in c2 c3 c4 c5 c1; do
NO_SQ=1 STEPS=200 bash tools/profile.sh $c ${1:-r06} || exit 1
done
NO_SQ=1 STEPS=200 bash tools/profile.sh c2 ${1:-r06} pyr || exit 1
}

# split probe on the GPU's NUMA node: pageable, pinned (runtime placement)
# and pinned with the thread's NUMA policy (hipHostMallocNumaUser), 3 rounds
step_p10() {
O=gpurun_out/r6p10
mkdir -p $O
g++ -O3 -std=c++20 -pthread -DWITH_HIP -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/split_probe.cpp -o $O/split_probe -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib || exit 1
NODE=$(timeout -k 10 120 python3 -c "
import torch
p = torch.cuda.get_device_properties(0)
a = '%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
print(open('/sys/bus/pci/devices/%s/numa_node' % a).read().strip())" 2>/dev/null)
[ -z "$NODE" ] || [ "$NODE" = "-1" ] && NODE=0
CPUS=$(cat /sys/devices/system/node/node$NODE/cpulist)
echo "node $NODE cpus $CPUS"
for rnd in 1 2 3; do
for k in pageable pinned pinned-numauser; do
timeout -k 10 120 taskset -c $CPUS $O/split_probe 128 $k split-nt,both-nt >> $O/split_probe.jsonl 2>&1 || { tail $O/split_probe.jsonl; exit 1; }
done
done
cat $O/split_probe.jsonl
}

# kernel + copy timelines of the e2e codec rows (tools/e2e_trace.sh,
# tools/timeline.py over the last 300 ms: the timed steps)
step_p11() {
bash tools/e2e_trace.sh r6z3 --steps 16 --warmup 4 --e2e pinned --codec zstd --clevel 3 || exit 1
python3 tools/timeline.py gpurun_out/e2e_r6z3/trace 300
bash tools/e2e_trace.sh r6bz2 --steps 16 --warmup 4 --e2e pinned --codec blosc-zstd --compress 2 || exit 1
python3 tools/timeline.py gpurun_out/e2e_r6bz2/trace 300
}

# compression streams: one per small level (default) vs the round-5 map
# (AQZ_COMP_STREAMS=2); codec tests first
step_p12() {
O=gpurun_out/r6p12
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_zstd.py -m gpu -q -x --timeout 100 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rnd in 1 2; do
for cs in 1 2; do
for a in "--codec zstd --clevel 3" "--codec blosc-zstd --compress 2" "--compress 1" "--codec zstd"; do
AQZ_COMP_STREAMS=$cs timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 --e2e pinned $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('r$rnd streams=$cs $a', d['value'], d.get('sink_bytes_per_input_byte'))"
done
done
done
}

"step_$@"
