#!/usr/bin/env bash
# Round-5 GPU runs, one function per gpurun call (the profiles/r05_* files
# come from these):  gpurun -- bash tools/r05_gpu.sh <step>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp

# probe rate vs launch size; the default bench line on the same box
step_p1() {
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 200 python3 -u tools/probe_sizes.py > $O/probe_sizes.jsonl 2> $O/probe.err || { tail $O/probe.err; exit 1; }
cat $O/probe_sizes.jsonl
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
}

# probe variants; placement tests; three default bench lines (fresh processes)
step_p2() {
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_sizes.py > $O/probe_variants.jsonl 2> $O/probe.err || { tail $O/probe.err; exit 1; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_placement.py -m gpu -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
for i in 1 2 3; do
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > $O/bench$i.json 2> $O/bench$i.err || { tail $O/bench$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench$i.json')); r=d['roofline']; p=r['placement']; print(json.dumps({'frac': r['frac'], 'ms': r['kernel_avg_ms'], 'cand': p['candidates_ms'], 'kept': p['kept'], 'exp': p['expected_ms'], 'probe': p['probe_bus_gbs'], 'acc': p['accepted'], 'peak_gb': round(p['peak_device_bytes']/1e9,2), 'est_gb': round(p['estimate_device_bytes']/1e9,2), 'ceil': r.get('probed_ceiling_same_shape')}))"
done
}

# candidates' stage time vs the streaming probe of the same memory
step_p3() {
O=gpurun_out/r5c
mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python3 -u tools/placement_r05.py --tries 6 >> $O/cand.jsonl 2>> $O/cand.err || { tail $O/cand.err; exit 1; }
timeout -k 10 120 python3 -u tools/placement_r05.py --tries 4 --plain >> $O/cand.jsonl 2>> $O/cand.err || { tail $O/cand.err; exit 1; }
done
timeout -k 10 120 python3 -u tools/placement_r05.py --tries 6 --batch 64 >> $O/cand.jsonl 2>> $O/cand.err || { tail $O/cand.err; exit 1; }
cat $O/cand.jsonl
}

# the whole GPU suite + smoke
step_full() {
O=gpurun_out/r5full
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
cat $O/smoke.log
}

# rocprof trace + PMC of the default bench line (tools/profile.sh)
step_prof() {
STEPS=200 bash tools/profile.sh ${1:-c2} ${2:-r05} || exit 1
}

# some GPU test files (names after the step)
step_tests() {
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest "$@" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -25 $O/pytest.log
[ $rc -eq 0 ] || exit 1
}

# C4 pair vs single-plane kernel: same-stage timing, PMC of each; C3 SQ/TA
step_p5() {
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,2 --instances 3 > $O/c4_knob_ab.txt 2>&1 || { tail $O/c4_knob_ab.txt; exit 1; }
cat $O/c4_knob_ab.txt
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
STEPS=200 bash tools/profile.sh c4 r05 || exit 1
STEPS=200 BENCH_EXTRA="--tune knobs=2" NAME_SUFFIX=-single bash tools/profile.sh c4 r05 || exit 1
STEPS=200 SQ2="TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU" bash tools/profile.sh c3 r05 || exit 1
}

# placement: stage vs probe over successive arenas; C4 write-request PMC
step_p6() {
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 200 python3 -u tools/placement_r05.py --config c4 --tries 3 --instances 5 >> $O/cand.jsonl 2>> $O/cand.err || { tail $O/cand.err; exit 1; }
timeout -k 10 200 python3 -u tools/placement_r05.py --config c2 --tries 3 --instances 4 >> $O/cand.jsonl 2>> $O/cand.err || { tail $O/cand.err; exit 1; }
cat $O/cand.jsonl
B="python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-pyramid-only-line --no-hbm-probe"
for v in 0 2; do
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_WRITE_SECTORS_sum --output-format csv -d $O/k$v-a -o run -- $B --tune knobs=$v > $O/k$v-a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_NORMAL_WRITEBACK_sum TCC_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_STREAMING_REQ_sum --output-format csv -d $O/k$v-b -o run -- $B --tune knobs=$v > $O/k$v-b.log 2>&1 || exit 1
done
}

# C4 pair kernel without spills: A/B, parity, PMC
step_p7() {
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,65536,2 --instances 3 > $O/c4_ab.txt 2>&1 || { tail $O/c4_ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --xy --knobs 0,65536 --instances 2 >> $O/c4_ab.txt 2>&1 || { tail $O/c4_ab.txt; exit 1; }
cat $O/c4_ab.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "3d or xy or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
NO_SQ=1 STEPS=200 bash tools/profile.sh c4 r05b || exit 1
}

# C3: launch size and occupancy A/Bs
step_p8() {
O=gpurun_out/r5h
mkdir -p $O
for B in 64 128; do
timeout -k 10 300 python3 -u tools/knob_ab.py --config c3 --batch $B --knobs 0,40960,49152,57344 --instances 2 >> $O/c3_ab.txt 2>&1 || { tail $O/c3_ab.txt; exit 1; }
done
cat $O/c3_ab.txt
}

# occupancy cap (unused LDS: v workgroups per CU) on every strip-kernel config
step_p9() {
O=gpurun_out/r5i
mkdir -p $O
for cfg in "c2 256" "c3 128" "c5 8" "c1 1024" "c2-ref4 128"; do
set -- $cfg
timeout -k 10 300 python3 -u tools/knob_ab.py --config $1 --batch $2 --knobs 0,40960,49152,57344 --instances 2 >> $O/cap_ab.txt 2>&1 || { tail $O/cap_ab.txt; exit 1; }
done
cat $O/cap_ab.txt
}

# bench lines of every config with the current build (device-resident)
step_lines() {
O=gpurun_out/r5lines${1:-}
mkdir -p $O
for c in c2 c3 c4 c5 c1 c2-ref4; do
timeout -k 10 200 python3 -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { tail $O/$c.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; p=r['placement']; print(json.dumps({'cfg': '$c', 'value': d['value'], 'frac': r['frac'], 'ms': r['kernel_avg_ms'], 'kernel': r['kernel'], 'cand': p.get('candidates_ms'), 'acc': p.get('accepted'), 'probe': r.get('probe_same_shape_gbs'), 'fop': r.get('frac_of_probe_same_shape'), 'traffic': r.get('traffic'), 'pyr': (d.get('pyramid_only') or {}).get('input_rate_frac_of_peak')}))" | tee -a $O/lines.jsonl
done
}

# end to end: the binding (pageable frames) and bench.py --e2e
step_e2e() {
O=gpurun_out/r5e2e
mkdir -p $O
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 --placement-tries 2 > $O/binding.jsonl 2> $O/binding.err || { tail $O/binding.err; exit 1; }
cat $O/binding.jsonl
for a in "--e2e pinned" "--e2e pinned --compress 1" "--e2e pinned --codec zstd" "--e2e pinned --codec zstd --clevel 3" "--e2e pinned --codec blosc-zstd --compress 2" "--e2e pageable"; do
timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 $a > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print(d['metric'][:60], d['value'], d.get('d2h_gbs_per_gpu'))"
done
}

# C4 pair kernel with next-pair prefetch: A/B and parity
step_p10() {
O=gpurun_out/r5p10
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,131072,2 --instances 3 > $O/c4_pf_ab.txt 2>&1 || { tail $O/c4_pf_ab.txt; exit 1; }
cat $O/c4_pf_ab.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "3d" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
}

# C4 launch size 128 vs 256 planes (prefetching pair kernel), and no-prefetch A/B
step_p11() {
O=gpurun_out/r5p11
mkdir -p $O
for B in 128 256; do
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --batch $B --knobs 0,131072 --instances 2 >> $O/c4_ab.txt 2>&1 || { tail $O/c4_ab.txt; exit 1; }
done
cat $O/c4_ab.txt
}

# C1 launch size; C5 and C1 PMC
step_p12() {
O=gpurun_out/r5p12
mkdir -p $O
for B in 1024 2048; do
timeout -k 10 300 python3 -u tools/knob_ab.py --config c1 --batch $B --knobs 0,8192 --instances 2 >> $O/c1_ab.txt 2>&1 || { tail $O/c1_ab.txt; exit 1; }
done
cat $O/c1_ab.txt
NO_SQ=1 STEPS=100 bash tools/profile.sh c5 r05 || exit 1
NO_SQ=1 STEPS=200 bash tools/profile.sh c1 r05 || exit 1
}

# C2 launch size 256 vs 512 frames; C2 profile of the shipped build
step_p13() {
O=gpurun_out/r5p13
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --batch 512 --knobs 0 --appends 256,512 --instances 2 >> $O/c2_ab.txt 2>&1 || { tail $O/c2_ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --batch 256 --knobs 0 --appends 128,256 --instances 2 >> $O/c2_ab.txt 2>&1 || { tail $O/c2_ab.txt; exit 1; }
cat $O/c2_ab.txt
STEPS=200 bash tools/profile.sh c2 r05d || exit 1
}

# C2 / C3 / C5 launch sizes on one stage
step_p14() {
O=gpurun_out/r5p14
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --batch 1024 --knobs 0 --appends 256,512,1024 --instances 2 --reps 10 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c3 --batch 512 --knobs 0 --appends 128,256,512 --instances 2 --reps 10 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c5 --batch 32 --knobs 0 --appends 8,16,32 --instances 2 --reps 10 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
cat $O/ab.txt
}

# the final build: GPU suite + smoke, every config's line, the default
# line, the C2 profile
step_final() {
step_full || exit 1
step_lines ${1:-f} || exit 1
O=gpurun_out/r5final
mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
STEPS=200 bash tools/profile.sh c2 ${2:-r05f} || exit 1
}

# final-build profiles of the other configs
step_profs() {
for c in c3 c4 c5 c1; do
STEPS=200 bash tools/profile.sh $c ${1:-r05f} || exit 1
done
}

# device zstd: the far-candidate pass (zstd_far) with buffer loads/stores
step_p16() {
O=gpurun_out/r5p16
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_zstd.py tests/test_gpu_codec.py -m gpu > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -3 $O/t.txt
bash tools/prof_zstd3.sh "--codec zstd --shuffle 0 --clevel 3" "--codec blosc-zstd --shuffle 2 --clevel 5" || exit 1
for a in "--clevel 3" "--clevel 1"; do
timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 --e2e pinned --codec zstd $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('$a', d['value'], d['ms_per_step'])"
done
}

# the shipped library after the zstd_far change: suite + smoke, C2 line + profile
step_final2() {
step_full || exit 1
O=gpurun_out/r5final2
mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
STEPS=200 bash tools/profile.sh c2 ${1:-r05g} || exit 1
}

# the shipped library: suite + smoke, default line, every configuration's profile
step_final3() {
step_full || exit 1
O=gpurun_out/r5final3
mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
for c in c2 c3 c4 c5 c1; do
STEPS=200 bash tools/profile.sh $c ${1:-r05h} || exit 1
done
}

# the shipped library: final3 (suite, default line, profiles), then the e2e rows
step_final4() {
step_final3 ${1:-r05i} || exit 1
step_e2e || exit 1
}

# e2e codec rows only (stream-priority A/B)
step_p17() {
O=gpurun_out/r5p17
mkdir -p $O
for a in "--e2e pinned --codec zstd --clevel 3" "--e2e pinned --codec blosc-zstd --compress 2" "--e2e pinned --compress 1" "--e2e pinned --codec zstd" "--e2e pinned"; do
timeout -k 10 200 python3 -u bench.py --steps 16 --warmup 4 $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
cat $O/tmp.json >> $O/bench_e2e.jsonl
python3 -c "import json; d=json.load(open('$O/tmp.json')); print('$a', d['value'], d['ms_per_step'], d.get('sink_bytes_per_input_byte'))"
done
}

"step_$@"
