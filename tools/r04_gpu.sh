#!/usr/bin/env bash
# Round-4 GPU runs, one function per gpurun call (the profiles/r04_* files
# came from these):  gpurun -- bash tools/r04_gpu.sh <step>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp

# knob tests + placement localisation (one process)
step_g1() {
mkdir -p gpurun_out/r4a
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "environment or 3d_shallow or xy_fused or async_handoff" > gpurun_out/r4a/pytest.log 2>&1 || { tail -30 gpurun_out/r4a/pytest.log; exit 1; }
tail -3 gpurun_out/r4a/pytest.log
timeout -k 10 300 python3 -u tools/placement_localize.py --trials 5 > gpurun_out/r4a/localize.jsonl 2> gpurun_out/r4a/localize.err || { tail gpurun_out/r4a/localize.err; exit 1; }
tail -2 gpurun_out/r4a/localize.jsonl
}

# placement localisation, one process per plan
step_g2() {
O=gpurun_out/r4b
mkdir -p $O
for plan in "start,src,src" "start,L=0x1e" "start,L=0x2,L=0x4,L=0x8,L=0x10" \
            "start,L=0x10,L=0x8,L=0x4,L=0x2" "pre=4096,start" "pre=16384,start" \
            "start,L=1,L=1,L=1" "start,all,all" "start,src,L=0x1e,L=1"; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --plan "$plan" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
cat $O/plans.jsonl
}

# contiguous vs hipMalloc ring sets
step_g3() {
O=gpurun_out/r4c
mkdir -p $O
for i in 1 2 3; do
for fl in 4 0; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --ring-flags $fl --plan "start,all,all,all,all" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
done
cat $O/plans.jsonl
}

# contiguous spacer sweep
step_g4() {
O=gpurun_out/r4d
mkdir -p $O
for S in 0 4 7 9 10.5 12 16 24 48 96 160; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --ring-flags 4 --spacer-gib $S --plan "start,all" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
for S in 12 48; do
  timeout -k 10 120 python3 -u tools/placement_localize.py --ring-flags 0 --spacer-gib $S --plan "start,all" >> $O/plans.jsonl 2>> $O/plans.err || { tail $O/plans.err; exit 1; }
done
cat $O/plans.jsonl
}

# placement search variants through bench.py
step_g5() {
O=gpurun_out/r4e
mkdir -p $O
run() { timeout -k 10 180 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line --no-hbm-probe "$@" > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/tmp.json')); r=d['roofline']; p=r['placement']; print(json.dumps({'args': sys.argv[1:], 'frac': r['frac'], 'ms': r['kernel_avg_ms'], 'cand': p['candidates_ms'], 'kept': p['kept'], 'peak_gb': round(p['peak_device_bytes']/1e9,2)}))" "$@" >> $O/runs.jsonl; }
run --placement-tries 16
run --placement-tries 16 --tune ring_malloc_flags=4
run --placement-tries 8 --tune placement_mode=1
run --placement-tries 8 --tune placement_mode=1 --tune ring_malloc_flags=4
run --placement-tries 16 --tune placement_spacer_bytes=1073741824
run --placement-tries 16 --tune placement_spacer_bytes=4294967296 --tune ring_malloc_flags=4
cat $O/runs.jsonl
}

# binding replay + golden tests, first binding timing
step_g6() {
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_handoff.py tests/test_gpu_golden.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -40 $O/pytest.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 -u tools/binding_e2e.py > $O/binding_e2e.jsonl 2> $O/binding_e2e.err || { tail $O/binding_e2e.err; exit 1; }
cat $O/binding_e2e.jsonl
}

# binding sweep (copy threads, slots, batch) vs bench e2e
step_g7() {
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
}

# binding rate vs bench.py e2e, same box
step_g8() {
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
}

# binding replay tests incl. z slabs
step_g9() {
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_handoff.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -30 $O/pytest.log
exit $rc
}

# placement search strategies, twice
step_g10() {
O=gpurun_out/r4j
mkdir -p $O
rm -f $O/runs.jsonl
run() { timeout -k 10 240 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line --no-hbm-probe "$@" > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/tmp.json')); r=d['roofline']; p=r['placement']; print(json.dumps({'args': sys.argv[1:], 'frac': r['frac'], 'ms': r['kernel_avg_ms'], 'c0': r.get('candidate0_ms'), 'kept': p['kept'], 'n': len(p['candidates_ms']), 'peak_gb': round(p['peak_device_bytes']/1e9,2)}))" "$@" >> $O/runs.jsonl; }
for rep in 1 2; do
run --placement-tries 16
run --placement-tries 16 --tune placement_spacer_bytes=2147483648
run --placement-tries 16 --tune placement_spacer_bytes=4294967296 --tune ring_malloc_flags=4
run --placement-tries 16 --tune placement_spacer_bytes=4294967296
run --placement-tries 12 --tune placement_mode=1 --tune ring_malloc_flags=4
done
cat $O/runs.jsonl
}

# strip kernel occupancy A/B
step_g11() {
O=gpurun_out/r4k
mkdir -p $O
K=0,$((2<<13)),$((3<<13)),$((4<<13)),$((5<<13)),$((6<<13))
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --knobs $K --instances 2 > $O/occ_ab2.txt 2>&1 || { tail $O/occ_ab2.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --knobs $K --instances 2 --placement-tries 16 >> $O/occ_ab2.txt 2>&1 || { tail $O/occ_ab2.txt; exit 1; }
cat $O/occ_ab2.txt
}

# 3-D parity incl. XY and pair kernels, C4 A/B
step_g12() {
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "3d or c4 or xy" > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,2,512 --instances 3 > $O/c4_ab.txt 2>&1 || { tail $O/c4_ab.txt; exit 1; }
cat $O/c4_ab.txt
timeout -k 10 300 python3 bench.py --config c4 --xy --steps 100 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > $O/c4xy.json 2> $O/c4xy.err || { tail $O/c4xy.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4xy.json')); r=d['roofline']; print('c4 xy', r['kernel'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'))"
}

# C4 pair kernel A/B on searched placements
step_g13() {
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,2,0,2 --instances 3 --placement-tries 16 > $O/c4_ab_search.txt 2>&1 || { tail $O/c4_ab_search.txt; exit 1; }
cat $O/c4_ab_search.txt
}

# full GPU suite + smoke + default bench
step_full() {
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
}

# round-4 rocprofv3 profiles + default bench
step_prof() {
# then the default bench line
NO_SQ=1 bash tools/profile.sh c2 r04 || exit 1
NO_SQ=1 bash tools/profile.sh c2 r04 pyr || exit 1
NO_SQ=1 bash tools/profile.sh c4 r04 || exit 1
mkdir -p gpurun_out/r4bench
timeout -k 10 600 python3 bench.py > gpurun_out/r4bench/bench_default.json 2> gpurun_out/r4bench/bench_default.err || { tail gpurun_out/r4bench/bench_default.err; exit 1; }
cat gpurun_out/r4bench/bench_default.json
}

# C4 pair profile and XY lines
step_prof2() {
# XY-transposed C2 / C4 bench lines against their live probes
NO_SQ=1 bash tools/profile.sh c4 r04b || exit 1
mkdir -p gpurun_out/r4xy
for c in c2 c4; do
  timeout -k 10 300 python3 bench.py --config $c --xy --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/r4xy/$c.json 2> gpurun_out/r4xy/$c.err || { tail gpurun_out/r4xy/$c.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --config c4 --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > gpurun_out/r4xy/c4_plain.json 2> gpurun_out/r4xy/c4p.err || { tail gpurun_out/r4xy/c4p.err; exit 1; }
for f in gpurun_out/r4xy/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$f', r['kernel'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'), r.get('candidate0_ms'))"; done
}

# C4 pair kernel: region walk order A/B (knob 1024 flips column-major)
step_g14() {
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,1024,2,0,1024 --instances 3 --placement-tries 16 > $O/c4_walk_ab.txt 2>&1 || { tail $O/c4_walk_ab.txt; exit 1; }
cat $O/c4_walk_ab.txt
}

# C2 strip kernel: chunk-major region walk (an experimental knob bit 31, since
# removed: 13-17% slower, profiles/r04_c2_walk_order_ab.txt) vs frame by frame
step_g15() {
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --knobs 0,2147483648,0,2147483648 --instances 2 > $O/c2_walk_ab.txt 2>&1 || { tail $O/c2_walk_ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --knobs 0,2147483648,0,2147483648 --instances 2 --placement-tries 16 >> $O/c2_walk_ab.txt 2>&1 || { tail $O/c2_walk_ab.txt; exit 1; }
cat $O/c2_walk_ab.txt
}

# XY-transposed storage order: row-major vs column-major region walk (knob
# 1024) on the fused XY loads
step_g16() {
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --xy --knobs 0,1024,0,1024 --instances 2 --placement-tries 16 > $O/xy_walk_ab.txt 2>&1 || { tail $O/xy_walk_ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --xy --knobs 0,1024,0,1024 --instances 2 --placement-tries 16 >> $O/xy_walk_ab.txt 2>&1 || { tail $O/xy_walk_ab.txt; exit 1; }
cat $O/xy_walk_ab.txt
}

# XY stages now run the placement search: exactness at the bench layout,
# then the XY bench lines (C2, C4) at the default search
step_g17() {
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_headline.py -k "c2_configuration" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -5 $O/pytest.txt
for c in c2 c4; do
timeout -k 10 240 python3 bench.py --config $c --xy --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > $O/xy_$c.json 2> $O/xy_$c.err || { tail $O/xy_$c.err; exit 1; }
tail -1 $O/xy_$c.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', d['value'], r['frac'], r.get('frac_of_probed_ceiling'), r['placement'].get('candidates_ms'), r['placement'].get('stage_create_s'), r['placement'].get('host_peak_rss_mib'))"
done
}

# XY on 2x2x2 pyramids, two planes at a time: parity, then the same-stage
# A/B against one plane at a time (knob 2), then the C4 --xy bench line
step_g18() {
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "xy_fused_strip3d" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --xy --knobs 0,2,0,2 --instances 3 --placement-tries 16 > $O/xy_pair_ab.txt 2>&1 || { tail $O/xy_pair_ab.txt; exit 1; }
cat $O/xy_pair_ab.txt
timeout -k 10 240 python3 bench.py --config c4 --xy --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line > $O/xy_c4.json 2> $O/xy_c4.err || { tail $O/xy_c4.err; exit 1; }
tail -1 $O/xy_c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c4', d['value'], r['kernel'], r['frac'], r.get('frac_of_probed_ceiling'), r['placement'].get('candidates_ms'))"
}

# build A/B: the previous library (acquire-zarr_amd/abx/libaqz_gpu_prev.so,
# region_xy through scratch) against the current one, alternating, each with
# its own placement search
step_g19() {
O=gpurun_out/r4s
mkdir -p $O
: > $O/lib_ab.txt
for c in c2 c4 c3; do
for rep in 1 2; do
for lib in prev cur; do
if [ $lib = prev ]; then export AQZ_LIB=$PWD/acquire-zarr_amd/abx/libaqz_gpu_prev.so; else unset AQZ_LIB; fi
timeout -k 10 240 python3 bench.py --config $c --steps 200 --warmup 5 --no-cpu-baseline --no-pyramid-only-line --no-hbm-probe > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
tail -1 $O/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=r['placement']; print('$c', '$lib', '$rep', round(r['achieved']/1e3*0+d['ms_per_step'],4), r['frac'], p.get('kept_ms_final'), min(p.get('candidates_ms') or [0]))" >> $O/lib_ab.txt
done
done
done
unset AQZ_LIB
cat $O/lib_ab.txt
}

# BASELINE configs[0] (C1, u16 512^2, 3 levels, decimate): the device-resident
# bench line with its CPU baseline, then the example end to end (raw and lz4,
# to shard files on the box's /tmp and without the sink)
step_g20() {
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 300 python3 bench.py --config c1 --steps 100 --warmup 5 > $O/c1.json 2> $O/c1.err || { tail $O/c1.err; exit 1; }
tail -2 $O/c1.json
for codec in raw lz4; do
for w in "--no-write" ""; do
rm -rf /tmp/aqz_c1
timeout -k 10 240 acquire-zarr_amd/examples/stream_to_filesystem /tmp/aqz_c1 --config c1 --frames 16384 --codec $codec --pattern camera $w >> $O/c1_e2e.jsonl 2> $O/c1_e2e.err || { tail $O/c1_e2e.err; exit 1; }
done
done
rm -rf /tmp/aqz_c1
cat $O/c1_e2e.jsonl
}

# the strip kernel for 0-2 fused levels (C1): parity, then the C1 bench line
step_g21() {
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "shallow_pyramid_strip or baseline_configs or xy_fused_strip or tile_split_and_pyramid or max_levels" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 300 python3 bench.py --config c1 --steps 100 --warmup 5 > $O/c1.json 2> $O/c1.err || { tail $O/c1.err; exit 1; }
tail -1 $O/c1.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c1', d['value'], r['kernel'], r['kernel_avg_ms'], r['frac'], r.get('frac_of_probed_ceiling'), d['pyramid_only']['kernel_input_frac_of_probed_ceiling'], d['cpu_baseline']['value'])"
}

# C1 on the strip kernel: kernel trace + PMC (traffic, SQ)
step_prof3() {
bash tools/profile.sh c1 r04 || exit 1
}

# placement: rings carved from one arena, moved inside it (tools/arena_probe.py)
step_g22() {
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 400 python3 -u tools/arena_probe.py --config c2 --stages 3 > $O/arena_c2.txt 2>&1 || { tail $O/arena_c2.txt; exit 1; }
timeout -k 10 300 python3 -u tools/arena_probe.py --config c2 --stages 2 --flags 0 >> $O/arena_c2.txt 2>&1 || { tail $O/arena_c2.txt; exit 1; }
grep -v amdgpu.ids $O/arena_c2.txt
}

# the arena probe at GiB offsets (16 GiB of slack)
step_g23() {
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 400 python3 -u tools/arena_probe.py --config c2 --stages 2 --slack-mib 16384 --offsets-kib 0,1048576,2097152,3145728,4194304,6291456,8388608,12582912,16777216 > $O/arena_gib.txt 2>&1 || { tail $O/arena_gib.txt; exit 1; }
timeout -k 10 300 python3 -u tools/arena_probe.py --config c2 --stages 1 --flags 0 --slack-mib 16384 --offsets-kib 0,1048576,2097152,3145728,4194304,6291456,8388608,12582912,16777216 >> $O/arena_gib.txt 2>&1 || { tail $O/arena_gib.txt; exit 1; }
grep -v amdgpu.ids $O/arena_gib.txt
}

# which translation (UTCL2 / TLB) counters this rocprofv3 offers
step_g24() {
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { tail $O/counters.txt; exit 1; }
grep -i -E "utc|tlb|translat|ATC|VM_|PTE|walk" $O/counters.txt | head -80
}

# slow vs fast placement: TCP->TCC request mix by memory type, and latencies
step_g25() {
O=gpurun_out/r4y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/mtype_probe.py > $O/plain.txt 2>&1 || { tail $O/plain.txt; exit 1; }
grep stage $O/plain.txt
i=0
for set in "TCP_TCC_RW_READ_REQ_sum TCP_TCC_NC_READ_REQ_sum TCP_TCC_CC_READ_REQ_sum TCP_TCC_UC_READ_REQ_sum" \
           "TCP_TCC_RW_WRITE_REQ_sum TCP_TCC_NC_WRITE_REQ_sum TCP_TCC_CC_WRITE_REQ_sum TCP_TCC_UC_WRITE_REQ_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
i=$((i+1))
timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- python3 tools/mtype_probe.py > $O/pmc$i.log 2>&1 || { tail $O/pmc$i.log; exit 1; }
grep stage $O/pmc$i.log
python3 tools/mtype_probe.py --summarise $O/pmc$i
done
}

# ring arena: exactness at moved offsets
step_g26() {
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "ring_arena or environment_cannot" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
}

# rings from the HIP virtual-memory API (hipMemCreate pieces mapped into one
# range; ring_malloc_flags 0x100 | log2(piece / granularity) << 9), no search
step_g27() {
O=gpurun_out/r4aa
mkdir -p $O
: > $O/vmm.txt
for rep in 1 2 3; do
for fl in 0 256 2304 4352 4864; do
timeout -k 10 200 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-pyramid-only-line --no-hbm-probe --placement-tries 0 --tune ring_malloc_flags=$fl > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
tail -1 $O/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('flags', $fl, 'rep', $rep, 'ms', d['ms_per_step'], 'kernel_ms', r['kernel_avg_ms'], 'frac', r['frac'])" >> $O/vmm.txt
done
done
cat $O/vmm.txt
}

# the VMM probe, bounded, large pieces first
step_g28() {
O=gpurun_out/r4ab
mkdir -p $O
for fl in 4864 4352 2304; do
timeout -k 10 90 python3 -u tools/vmm_probe.py --flags $fl >> $O/vmm.txt 2>&1 || { tail $O/vmm.txt; exit 1; }
done
grep -v amdgpu.ids $O/vmm.txt
}

# VMM rings vs plain hipMalloc, first allocation of each process, 3 reps
step_g29() {
O=gpurun_out/r4ac
mkdir -p $O
for rep in 1 2 3; do
for fl in 0 4864 4352 5376; do
echo "rep $rep" >> $O/vmm.txt
timeout -k 10 90 python3 -u tools/vmm_probe.py --flags $fl --launches 50 >> $O/vmm.txt 2>&1 || { tail $O/vmm.txt; exit 1; }
done
done
grep -v amdgpu.ids $O/vmm.txt | paste - - - - - | awk '{print $2, $4, $NF-0, $(NF-1)}'
}

# VMM rings: one piece per ring (exact size) vs 1 GiB pieces vs hipMalloc,
# on C2, C4, C3, C5, C1
step_g30() {
O=gpurun_out/r4ad
mkdir -p $O
for cfg in c2 c4 c3 c5 c1; do
for rep in 1 2; do
for fl in 0 7936 4864; do
echo "$cfg rep $rep" >> $O/vmm.txt
timeout -k 10 90 python3 -u tools/vmm_probe.py --config $cfg --flags $fl --launches 50 >> $O/vmm.txt 2>&1 || { tail $O/vmm.txt; exit 1; }
done
done
done
grep -v amdgpu.ids $O/vmm.txt | paste - - - - - | awk '{print $1, $3, $5, $(NF-1)}'
}

# VMM pieces with every ring packed into one arena (512 MiB / 1 GiB pieces)
step_g31() {
O=gpurun_out/r4ae
mkdir -p $O
for cfg in c2 c4 c3 c5 c1; do
for fl in 4352 4864; do
echo "$cfg" >> $O/vmm.txt
timeout -k 10 90 python3 -u tools/vmm_probe.py --config $cfg --flags $fl --arena 4096 --launches 50 >> $O/vmm.txt 2>&1 || { tail $O/vmm.txt; exit 1; }
done
done
grep -v amdgpu.ids $O/vmm.txt | paste - - - - - | awk '{print $1, $3, $5, $(NF-1)}'
}

# the shipped VMM arena inside bench.py (with / without the HBM probe and the
# pyramid-only side run) against the standalone probe
step_g32() {
O=gpurun_out/r4af
mkdir -p $O
: > $O/arena_bench.txt
for rep in 1 2; do
for mode in plain noprobe default; do
case $mode in
plain) A="--no-cpu-baseline --no-pyramid-only-line --no-hbm-probe --tune ring_malloc_flags=65536";;
noprobe) A="--no-cpu-baseline --no-pyramid-only-line --no-hbm-probe";;
default) A="--no-cpu-baseline";;
esac
timeout -k 10 200 python3 bench.py --steps 100 --warmup 5 $A > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
tail -1 $O/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$mode', $rep, d['ms_per_step'], r['kernel_avg_ms'], r['placement']['candidates_ms'], r['placement']['mode'])" >> $O/arena_bench.txt
done
timeout -k 10 90 python3 -u tools/vmm_probe.py --flags 0 --launches 50 >> $O/arena_bench.txt 2>&1 || { tail $O/arena_bench.txt; exit 1; }
done
grep -v amdgpu.ids $O/arena_bench.txt
}

# VMM arena piece size sweep (pieces of 2^(16+v) bytes: v = 5 2 MiB, 6 4 MiB,
# 7 8 MiB, 8 16 MiB, 10 64 MiB), hipMalloc per level (65536) as control
step_g33() {
O=gpurun_out/r4ag
mkdir -p $O
: > $O/pieces.txt
for rep in 1 2; do
for cfg in c2 c3 c4; do
for fl in 65536 2816 3328 3840 4352 5376; do
A="--arena 4096"; [ $fl = 65536 ] && A=""
echo "$cfg" >> $O/pieces.txt
timeout -k 10 90 python3 -u tools/vmm_probe.py --config $cfg --flags $fl $A --launches 50 >> $O/pieces.txt 2>&1 || { tail $O/pieces.txt; exit 1; }
done
done
done
grep -v amdgpu.ids $O/pieces.txt | paste - - - - - | awk '{print $1, $3, $7, $(NF-1)}'
}

# every configuration's bench line with the shipped ring arena (one box)
step_g34() {
O=gpurun_out/r4ah
mkdir -p $O
: > $O/lines.jsonl
for a in "--config c1" "--config c2" "--config c2-ref4" "--config c3" "--config c4" "--config c5" "--config c2 --xy" "--config c4 --xy"; do
timeout -k 10 300 python3 bench.py $a --steps 200 --warmup 5 --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
tail -1 $O/tmp.json >> $O/lines.jsonl
tail -1 $O/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$a', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_of_probed_ceiling'), r['placement']['candidates_ms'], d.get('pyramid_only',{}).get('kernel_input_frac_of_probed_ceiling'))"
done
}

# rocprofv3 trace + PMC of C2, C2 pyramid-only and C4 with the shipped arena
step_prof4() {
NO_SQ=1 bash tools/profile.sh c2 r04v || exit 1
NO_SQ=1 bash tools/profile.sh c2 r04v pyr || exit 1
NO_SQ=1 bash tools/profile.sh c4 r04v || exit 1
}

# successive arenas in one process (earlier ones held), 3 processes; plain too
step_g35() {
O=gpurun_out/r4ai
mkdir -p $O
for rep in 1 2 3; do
timeout -k 10 120 python3 -u tools/arena_multi.py --stages 4 >> $O/multi.txt 2>&1 || { tail $O/multi.txt; exit 1; }
done
timeout -k 10 120 python3 -u tools/arena_multi.py --stages 4 --flags 65536 >> $O/multi.txt 2>&1 || { tail $O/multi.txt; exit 1; }
grep -v amdgpu.ids $O/multi.txt
}

# e2e codec rows with the ring arena (pinned frames), against round 3's
step_g36() {
O=gpurun_out/r4aj
mkdir -p $O
: > $O/e2e.jsonl
for a in "--codec none" "--codec lz4 --compress 2" "--codec blosc-zstd --compress 1" "--codec blosc-zstd --compress 2" "--codec zstd" "--codec zstd --clevel 3"; do
timeout -k 10 240 python3 bench.py --steps 16 --warmup 2 --e2e pinned $a > $O/tmp.log 2>&1 || { tail -20 $O/tmp.log; exit 1; }
grep '^{' $O/tmp.log | tail -1 >> $O/e2e.jsonl
grep '^{' $O/tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'])"
done
}

# e2e codec rows: codec / staging buffers from hipMalloc vs 2 MiB pieces
# (zstd_flags bit 20), alternating
step_g37() {
O=gpurun_out/r4ak
mkdir -p $O
: > $O/e2e_vmm.txt
for a in "--codec zstd --clevel 3" "--codec blosc-zstd --compress 2" "--codec lz4 --compress 2"; do
for v in 0 1048576 0 1048576; do
timeout -k 10 240 python3 bench.py --steps 16 --warmup 2 --e2e pinned $a --tune zstd_flags=$v > $O/tmp.log 2>&1 || { tail -20 $O/tmp.log; exit 1; }
grep '^{' $O/tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', 'zstd_flags=$v', d['value'], d['ms_per_step'])" >> $O/e2e_vmm.txt
done
done
cat $O/e2e_vmm.txt
}

# the live HBM probe with hipMalloc'd vs 2 MiB-piece buffers, alternating
step_g38() {
O=gpurun_out/r4al
mkdir -p $O
timeout -k 10 200 python3 -u - > $O/probe_pieces.txt 2>&1 <<'PY' || { tail $O/probe_pieces.txt; exit 1; }
import sys
sys.path.insert(0, "acquire-zarr_amd")
import aqz
names = {aqz.PROBE_READ: "read", aqz.PROBE_COPY: "copy", aqz.PROBE_COPY_THIRD: "copy+1/3",
         aqz.PROBE_READ_THIRD: "read+1/3"}
wr = {aqz.PROBE_READ: 0.0, aqz.PROBE_COPY: 1.0, aqz.PROBE_COPY_THIRD: 4 / 3,
      aqz.PROBE_READ_THIRD: 1 / 3}
for rnd in range(3):
    for shape in names:
        row = []
        for pc in (0, aqz.PROBE_PIECES):
            best = 0.0
            for st in (0, aqz.PROBE_PLAIN_STORES) if shape != aqz.PROBE_READ else (0,):
                ms, rd = aqz.probe_hbm(shape | st | pc, 512 << 20, 20, 0)
                best = max(best, rd * (1 + wr[shape]) / (ms * 1e-3) / 1e9)
            row.append(round(best, 1))
        print(rnd, names[shape], "hipMalloc", row[0], "pieces", row[1], "GB/s", flush=True)
PY
cat $O/probe_pieces.txt
}

# the drop-in binding end to end with the ring arena (handoff_replay)
step_g39() {
O=gpurun_out/r4am
mkdir -p $O
timeout -k 10 400 python3 -u tools/binding_e2e.py --frames 2048 > $O/binding_e2e.jsonl 2> $O/binding_e2e.err || { tail $O/binding_e2e.err; exit 1; }
cat $O/binding_e2e.jsonl
}

# kernel A/Bs on the ring arena: C4 pair vs one plane (XY and not), C3 and
# C2 occupancy caps (knob bits 13-15 = workgroups per CU)
step_g40() {
O=gpurun_out/r4an
mkdir -p $O
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --xy --knobs 0,2,0,2 --instances 2 > $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c4 --knobs 0,2,0,2 --instances 2 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c3 --knobs 0,40960,49152,57344 --instances 2 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
timeout -k 10 300 python3 -u tools/knob_ab.py --config c2 --knobs 0,40960,49152,57344 --instances 2 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
}

# the default bench three times (hybrid placement), then C3 and C4
step_g41() {
O=gpurun_out/r4ao
mkdir -p $O
: > $O/lines.jsonl
for a in "--config c2" "--config c2" "--config c2" "--config c3" "--config c4"; do
timeout -k 10 300 python3 bench.py $a --no-cpu-baseline > $O/tmp.json 2> $O/tmp.err || { tail $O/tmp.err; exit 1; }
tail -1 $O/tmp.json >> $O/lines.jsonl
tail -1 $O/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=r['placement']; print('$a', d['value'], d['ms_per_step'], r['frac'], r.get('frac_of_probed_ceiling'), p['candidates_ms'], p['kept'], round(p['peak_device_bytes']/1e9,1))"
done
}

"step_$1"
