/*
 * aqz_gpu_bench.h -- measurement and tuning entry points of libaqz_gpu.so.
 *
 * NOT part of the drop-in ABI (include/aqz_gpu.h): nothing the reference's
 * streaming layer calls.  bench.py, the tuning tools under tools/ and the
 * tests use these to reproduce the BASELINE configurations and to time the
 * dominant kernel on the stream it runs on.
 */
#ifndef AQZ_GPU_BENCH_H
#define AQZ_GPU_BENCH_H

#include "aqz_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct
{
    uint32_t force_levels;     /* 0 = the reference level rule
                                  (downsampler.cpp:512-541).  >0: keep halving
                                  XY until this many levels exist -- BASELINE
                                  configs[1] asks for 5 levels at 256-px
                                  chunks, where the rule stops at 4; pixels
                                  are unchanged (each level is the 2x2 of the
                                  one above). */
    int32_t skip_level0_split; /* 1 = do not tile-split level 0 (the
                                  pyramid-only side measurement) */
    uint32_t placement_tries;  /* creation-time placement search: 0 = the
                                  aqz_stage_options value; n > 1 = as there
                                  (aqz_stage_options.placement_tries) */
    uint32_t placement_reps;   /* timed launches per candidate (0 = 10) */
    uint32_t placement_flags;  /* 1: never accept a candidate against the
                                  probe's expectation (every try runs: the
                                  search's worst-case peak, for tests) */
    /* Kernel tuning for A/B runs.  The library reads none of these from the
     * environment: a stage made by aqz_stage_create always runs the shipped
     * kernels.  Knob bits that skip stores (timing experiments only) exist
     * only here. */
    uint32_t knobs;            /* kernel A/B switches (0 = shipped kernels) */
    uint32_t nt_policy;        /* 0 = shipped (7); 8 | p = nontemporal policy p
                                  (bit 0 input loads, 1 level-0 stores,
                                  2 level-1/2 stores) */
    uint32_t xcd_rot;          /* regions each XCD's walk is rotated by */
    uint32_t region_rows_log2; /* 0 = automatic */
    uint32_t zstd_flags;       /* device zstd encoder A/B (frames still decode):
                                  1 literals only (no LZ matches: the serial
                                  model's byte-exact mode), 2 no far
                                  candidates, 4 predefined sequence tables
                                  only; bits 8-15 the parse history, bits
                                  16-19 parse variants; bit 20: codec work
                                  buffers, layer frames and H2D staging of
                                  >= 64 MiB from 2 MiB virtual-memory
                                  pieces, as the rings; bit 21: the far
                                  pass walks every segment as one range */
    uint32_t ring_malloc_flags; /* 0 = shipped: rings of >= 256 MiB in all
                                   are packed into one arena of 2 MiB
                                   virtual-memory pieces (hipMemCreate +
                                   hipMemMap), smaller ones hipMalloc'd.
                                   Otherwise per-level rings (the round-3
                                   placement, for A/B): hipExtMallocWithFlags
                                   flags, 0x10000 alone = hipMalloc, 0x100 |
                                   v << 9 = virtual memory in pieces of
                                   2^(16 + v) bytes (v = 31: one piece of the
                                   ring's own size).  With ring_arena_bytes
                                   the arena takes these flags. */
    uint64_t chunk_pad_bytes;  /* device bytes added between the chunks of a
                                  resident layer (chunk_pitch) */
    uint64_t ring_spacer_bytes; /* a device allocation (ring_malloc_flags) made
                                   before the rings and freed after them */
    uint64_t ring_arena_bytes;  /* > 0: every level's ring is carved from ONE
                                   allocation (ring_malloc_flags) with this much
                                   slack, movable by
                                   aqz_stage_bench_set_ring_offset; no
                                   placement search */
} aqz_stage_bench_options;

/* aqz_stage_estimate_memory including the placement search's transient
 * creation peak (bench may be NULL = aqz_stage_estimate_memory). */
aqz_status aqz_stage_estimate_memory_bench(const aqz_array_desc* desc,
                                           const aqz_stage_options* opt,
                                           const aqz_stage_bench_options* bench,
                                           aqz_memory_usage* out);

/* What the placement search did. */
typedef struct
{
    uint32_t n;                 /* candidates timed (0 = no search ran) */
    uint32_t kept;              /* index of the kept one */
    uint32_t reps;              /* timed launches per candidate (random frames) */
    uint32_t mode;              /* 3: ring arenas of 2 MiB pieces, 4: per-level
                                   ring allocations */
    double ms[32];              /* ms per launch, candidates 0..min(n,32)-1 */
    double kept_ms_final;       /* the kept placement re-timed alone, after
                                   the others were freed */
    uint64_t peak_device_bytes; /* the stage's device bytes at the search's peak */
    double probe_bus_gbs;       /* the probe of the stage's bus shape -- copy-
                                   third (1 read : 4/3 write), or read-third
                                   (1 : 1/3) without the level-0 split --
                                   streaming the random frames into the first
                                   candidate's memory, bus GB/s (0 = not run) */
    double expected_ms;         /* alg_bytes at probe_bus_gbs */
    uint64_t alg_bytes;         /* algorithmic bytes of one timing launch */
    uint32_t accepted;          /* 1: the kept candidate is within 3% of
                                   expected_ms (the search stopped there) */
    uint32_t stop;              /* why the search stopped: 1 accepted, 2 every
                                   try ran, 3 no expectation (the probe's
                                   source or memory too small), 4 out of
                                   memory (the best so far kept) */
    double probe_gbs[32];       /* the probe over each candidate's memory */
} aqz_placement_report;
aqz_status aqz_stage_placement_report(const aqz_stage* st, aqz_placement_report* out);

/* aqz_stage_create with the bench extensions (bench may be NULL). */
aqz_status aqz_stage_create_bench(const aqz_array_desc* desc,
                                  const aqz_stage_options* opt,
                                  const aqz_stage_bench_options* bench,
                                  aqz_stage** out);

/* Kernel A/B switches for tuning runs (0, 0 = the shipped kernels). */
aqz_status aqz_stage_set_tuning(aqz_stage* st, uint32_t knobs, uint32_t nt);

/* Placement experiments: allocate fresh chunk-layer rings (with their
 * has_data words and frame tables) for the levels whose bit is set in
 * level_mask; the old ones stay allocated until the stage is destroyed, so
 * the new ones land in other memory.  Ring contents are lost (timing only). */
aqz_status aqz_stage_bench_replace_rings(aqz_stage* st, uint32_t level_mask);

/* ring_arena_bytes stages: move every level's ring to arena + offset bytes
   (levels back to back, each 64 KiB aligned; offset a multiple of 256 and
   within the slack).  Synchronises the stage, re-zeroes the rings and
   restarts it at frame 0 (what was written is dropped). */
aqz_status aqz_stage_bench_set_ring_offset(aqz_stage* st, uint64_t offset);

/* Time every launch of the dominant (fused pyramid) kernel with HIP events
 * recorded on the stream it is launched on. */
aqz_status aqz_stage_enable_kernel_timing(aqz_stage* st, int32_t enable);
/* Sum of those kernels' durations (ms) and their count since enabling;
 * synchronizes. */
aqz_status aqz_stage_kernel_timing(aqz_stage* st, double* total_ms,
                                   uint64_t* launches);
/* One timing event pair on the stage's stream (the stream its kernels run
 * on): which = 0 records the begin mark, 1 the end mark, after all work
 * enqueued so far.  aqz_stage_timing_elapsed waits for the end mark and
 * returns the milliseconds between the two. */
aqz_status aqz_stage_timing_mark(aqz_stage* st, int32_t which);
aqz_status aqz_stage_timing_elapsed(aqz_stage* st, double* ms);
/* Name of the dominant kernel symbol (for matching rocprof output). */
const char* aqz_stage_dominant_kernel(const aqz_stage* st);
/* Ranges the device zstd far pass walked each segment of `level`'s last
 * compressed layer in (1 = one sequential walk; 0 = no far pass or no
 * compression yet): the ranges follow from the layer geometry alone. */
uint32_t aqz_stage_zstd_far_ranges(const aqz_stage* st, uint32_t level);

/* Placement calibration done at creation (the chunk-layer rings were
 * allocated up to n times and the fastest placement kept): the ms per
 * calibration launch of every candidate (up to cap of them, *n = count,
 * 0 = no calibration ran) and the index of the one kept. */
aqz_status aqz_stage_placement(const aqz_stage* st, double* ms, size_t cap,
                               size_t* n, uint32_t* kept);

/* NUMA placement of the stage's host threads (staging copy pool, host zstd
 * pool): the NUMA node of the stage's device (-1 = unknown) and how many of
 * this process's CPUs lie on it (0 = the threads are not pinned). */
aqz_status aqz_stage_host_affinity(const aqz_stage* st, int32_t* numa_node,
                                   uint32_t* n_cpus);

/* Streaming probe of this device's practical HBM rates, for the access
 * shapes the stage runs ("verify on the box with a read-only
 * stream kernel, and report the measured practical peak").  Every
 * workgroup streams one contiguous 24 KiB block with 16-B lane accesses
 * (nontemporal loads, nontemporal stores) over a source ring of 4 x bytes:
 *   AQZ_PROBE_READ         read only
 *   AQZ_PROBE_COPY         1 read : 1 write
 *   AQZ_PROBE_COPY_THIRD   1 read : 4/3 write (the full stage)
 *   AQZ_PROBE_READ_THIRD   1 read : 1/3 write (the pyramid-only stage)
 * | AQZ_PROBE_PLAIN_STORES: plain instead of nontemporal stores (which of
 * the two is faster depends on the shape; a ceiling is the better one).
 * ms = mean launch time over reps launches (after 3 warm-ups) on device
 * `device`; read_bytes = bytes read per launch (<= bytes).  Allocates and
 * frees ~6 x bytes of device memory. */
enum
{
    AQZ_PROBE_READ = 0,
    AQZ_PROBE_COPY = 1,
    AQZ_PROBE_COPY_THIRD = 2,
    AQZ_PROBE_READ_THIRD = 3,
    AQZ_PROBE_PLAIN_STORES = 0x100,
    AQZ_PROBE_PIECES = 0x200, /* buffers from 2 MiB virtual-memory pieces, as
                                 the stage's chunk-layer rings */
    AQZ_PROBE_DEEP = 0x400    /* 192 B per lane in flight (48 KiB per
                                 workgroup) instead of 96 B */
};
aqz_status aqz_probe_hbm(int32_t device, int32_t shape, uint64_t bytes, uint32_t reps,
                         double* ms, uint64_t* read_bytes);

#ifdef __cplusplus
}
#endif
#endif /* AQZ_GPU_BENCH_H */
