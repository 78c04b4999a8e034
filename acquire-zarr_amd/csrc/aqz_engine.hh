// aqz_engine.hh -- host engine of the MI355X multiscale stage.
//
//   Stage          <- the hot path of zarr::MultiscaleArray::write_frame
//                     (src/streaming/multiscale.array.cpp:57-74, 291-325):
//                     level-0 tile split + Downsampler::add_frame + tile split
//                     of every level, batched and device-resident.
//   GpuDownsampler <- zarr::Downsampler (src/streaming/downsampler.hh:12-64),
//                     same add_frame/take_frame contract.
#pragma once

#include "aqz_codec.hh"
#include "aqz_copy.hh"
#include "aqz_geometry.hh"
#include "aqz_hostsplit.hh"
#include "aqz_hostzstd.hh"
#include "aqz_params.hh"

#include <hip/hip_runtime.h>
#include <hsa/hsa.h>

#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace aqz {

hipError_t launch_fused_pyramid(int dtype, int method, const FusedParams& p,
                                hipStream_t stream);
hipError_t launch_level(int dtype, int method, const LevelParams& p,
                        hipStream_t stream);
hipError_t launch_fused_pyramid_3d(int dtype, int method, const FusedParams& p,
                                   hipStream_t stream);
hipError_t launch_transpose_frames(const void* src, void* dst, uint32_t rows,
                                   uint32_t cols, uint32_t n_frames, uint32_t bpp,
                                   hipStream_t stream);
hipError_t launch_flags_to_bytes(const uint32_t* flags, uint8_t* out, uint32_t n,
                                 uint32_t tag, hipStream_t stream);
hipError_t launch_fill_random(void* p, uint64_t bytes, uint64_t seed, hipStream_t stream);
hipError_t launch_import_frames(uint8_t* dst, const uint8_t* src, const uint64_t* tab_off,
                                const uint32_t* tab_grp, uint32_t f0, uint32_t n_frames,
                                uint32_t n_tiles, uint64_t pitch, uint32_t tile_bytes,
                                uint32_t* dst_flags, const uint32_t* src_flags, uint32_t tag,
                                hipStream_t stream);
hipError_t launch_zero_frame_tiles(uint8_t* fb, uint64_t bpc,
                                   uint32_t n_tiles, uint32_t tile_bytes,
                                   hipStream_t stream);
// aqz_probe.hip: the copy-third streaming shape (1 read : 4/3 write) of
// read_bytes from src into dst (>= 4/3 read_bytes + one workgroup's block),
// variant 0-2 (kPlacementProbeVariants); third_only: the read-third shape
// (1 read : 1/3 write) of a stage without the level-0 split.  The largest
// read size a source and destination of these sizes take (0 = too small)
constexpr int kPlacementProbeVariants = 3;
uint64_t probe_copy_third_read_bytes(uint64_t src_bytes, uint64_t dst_bytes);
hipError_t launch_probe_copy_third(const uint8_t* src, uint8_t* dst, uint64_t read_bytes,
                                   hipStream_t stream, int variant, bool third_only = false);

void hip_check(hipError_t e, const char* what);

// Owning device allocation (or, after set_view, a non-owning view into
// another one).
struct DevBuf
{
    uint8_t* p = nullptr;
    size_t n = 0;
    bool view = false;
    // kVmm allocations (the ring arena): physical pieces of vmm_piece bytes
    // from hipMemCreate, the first vmm_mapped of them mapped back to back
    // into one reserved range of vmm_span bytes.  vmm_span != 0 marks a
    // reserved range (released piece by piece, never hipFree'd).
    std::vector<hipMemGenericAllocationHandle_t> vmm;
    size_t vmm_span = 0;
    size_t vmm_piece = 0;
    size_t vmm_mapped = 0;
    static constexpr unsigned kVmm = 0x100u; // alloc flag; bits 9-13 = v:
                                             // pieces of 2^(16 + v) bytes
                                             // (31: the whole size)
    size_t physical() const { return vmm_span ? vmm_span : n; }
    DevBuf() = default;
    explicit DevBuf(size_t bytes) { alloc(bytes); }
    ~DevBuf();
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept;
    DevBuf& operator=(DevBuf&& o) noexcept;
    // flags: hipExtMallocWithFlags flags (0 = hipMalloc)
    void alloc(size_t bytes, unsigned flags = 0);
    // [q, q + bytes) of an allocation someone else owns (and frees)
    void set_view(uint8_t* q, size_t bytes);
    void release();
};

// Owning pinned host allocation.
struct PinnedBuf
{
    uint8_t* p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    ~PinnedBuf();
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    PinnedBuf(PinnedBuf&& o) noexcept
      : p(o.p)
      , n(o.n)
    {
        o.p = nullptr;
        o.n = 0;
    }
    void alloc(size_t bytes);
};

// Chunk compression settings (ZarrCompressionSettings, zarr.types.h:112-122;
// codec values of ZarrCompressionCodec).
struct Compression
{
    int32_t codec = 0;   // 0 none, 1 blosc-lz4, 2 blosc-zstd, 3 zstd
    int32_t clevel = 1;  // blosc clevel (0 stores every chunk uncompressed);
                         // zstd level (the device encoder: zstd_far_slices)
    int32_t shuffle = 1; // 0 none, 1 byte, 2 bit
};

// A/B switches of the device zstd encoder (aqz_stage_bench_options): every
// setting still writes frames that decode to the chunk bytes.
struct CodecTuning
{
    uint32_t match = 1;    // 0: literals only (the serial model's byte-exact mode)
    uint32_t far = 1;      // 0: no far candidates
    uint32_t fit = 1;      // 0: predefined sequence tables only
    uint32_t phist = 0;    // parse history (KiB before a unit; 0 none)
    uint32_t parse = 0;    // parse variants for timing (bits 1/2/4/8)
    uint32_t vmm = 0;      // 1: buffers >= 64 MiB (codec work buffers, layer
                           // frames, H2D staging) from 2 MiB virtual-memory
                           // pieces, as the rings (A/B)
    uint32_t ranges = 1;   // 0: the far pass walks every segment as one range
};

// Device frames of arrays of equally sized device chunks (aqz_codec.hip):
// blosc1-lz4, blosc1-zstd or plain zstd.
// hash slices of the device zstd far-candidate pass (0: none); aqz_engine.cpp
uint32_t zstd_far_slices(const Compression& c, uint32_t typesize);

class Compressor
{
  public:
    Compressor(uint64_t chunk_bytes, uint32_t typesize, const Compression& c,
               const CodecTuning& tune = CodecTuning{});
    // bytes that always hold the frames of n_chunks chunks (any codec).
    // blosc frames never pass nbytes + 16 (the memcpyed rule); a plain zstd
    // frame of incompressible data is its header (<= 13 B) plus one raw
    // block (3-B header) per zstd::kBlock of input.
    static uint64_t max_bytes(uint64_t chunk_bytes, uint32_t n_chunks)
    {
        return uint64_t(n_chunks) *
               (chunk_bytes + 32 + 3 * (chunk_bytes / zstd::kBlock + 1));
    }
    // Enqueue on `stream`: the frames of n_chunks chunks (chunk i at
    // chunks + i * pitch; skipped unless flags[i] == tag when flags is
    // given) back to back into out; offsets (device, n_chunks + 1 words)
    // gets each frame's start and the total.
    // order (device, optional): output position -> chunk.
    void run(const uint8_t* chunks, uint64_t pitch, uint32_t n_chunks,
             const uint32_t* flags, uint32_t tag, uint8_t* out, uint64_t* offsets,
             hipStream_t stream, const uint32_t* order = nullptr);
    const BloscGeom& geom() const { return g_; }
    // bytes of one plane (a frame's tile) of a chunk: the far pass's ranged
    // walk warms up over at least two of them (0: unknown)
    void set_plane_bytes(uint64_t b) { plane_bytes_ = b; }
    uint64_t chunk_bytes() const { return nbytes_; }
    // ranges of the last run's far pass (0: none ran)
    uint32_t far_ranges() const { return far_ranges_; }
    // the blosc block size recorded in the frames (0: plain zstd)
    uint32_t blocksize() const
    {
        if (c_.codec == 1)
            return g_.blocksize;
        if (c_.codec == 2)
            return make_zstd_blosc_geom(uint32_t(nbytes_), typesize_).blocksize;
        return 0;
    }
    // device bytes of the scratch buffers run() allocates for n_chunks
    // chunks of chunk_bytes (an upper bound: aqz_compressor_scratch_bytes)
    static uint64_t scratch_bytes(const Compression& c, uint64_t chunk_bytes,
                                  uint32_t typesize, uint32_t n_chunks);
    // device bytes of the scratch buffers allocated so far
    uint64_t device_bytes() const
    {
        uint64_t n = scratch_.n + ssize_.n + spos_.n + fsize_.n + mode_.n + cstart_.n;
        for (const DevBuf* b : { &zin_, &hist_, &scount_, &bkind_, &bpay_, &bpos_, &tab_, &carrier_,
                                 &sraw_, &lits_, &seqs_, &snseq_, &snlit_, &stail_, &bltype_,
                                 &bnseq_, &sqt_, &scarrier_, &sval_,
                                 &bseqb_, &bnlit_, &seqt_, &far_ })
            n += b->n;
        return n;
    }

  private:
    void run_zstd(const uint8_t* chunks, uint64_t pitch, uint32_t n_chunks,
                  const uint32_t* flags, uint32_t tag, uint8_t* out, uint64_t* offsets,
                  hipStream_t stream, const uint32_t* order);
    Compression c_;
    CodecTuning tune_;
    uint64_t nbytes_ = 0;
    uint64_t plane_bytes_ = 0;
    uint32_t far_ranges_ = 0;
    uint32_t typesize_ = 1;
    BloscGeom g_{};
    bool store_only_;
    DevBuf scratch_, ssize_, spos_, fsize_, mode_, cstart_;
    DevBuf zin_, hist_, scount_, bkind_, bpay_, bpos_, tab_, carrier_, sraw_; // zstd
    DevBuf bnseq_, sqt_, scarrier_, sval_;
    DevBuf lits_, seqs_, snseq_, snlit_, stail_, bltype_, bseqb_, bnlit_, seqt_, far_;
};

struct ArrayDesc
{
    std::vector<Dim> dims; // acquisition order
    int32_t dtype = 0;
    bool multiscale = true;
    int32_t method = 0;
    uint32_t max_levels = 0;
    std::vector<size_t> storage_order;
    int32_t device = 0;
};

// StageOptions::ring_malloc_flags bit: per-level ring allocations (the
// round-3 placement) instead of the shipped arena
constexpr uint32_t kRingsPlain = 0x10000u;

struct StageOptions
{
    uint32_t layer_slots = 2;
    uint32_t max_batch_frames = 64;
    uint32_t force_levels = 0;
    bool skip_level0_split = false;
    // aqz_stage_options.level0_split_on_host: no level-0 split on the device
    // (implies skip_level0_split); the caller splits level 0 on the host
    bool level0_on_host = false;
    uint64_t first_frame = 0;
    uint32_t z_slab_begin = 0, z_slab_end = 0; // aqz_stage_options
    // creation-time placement search (aqz_stage_options.placement_tries;
    // 0/1 = off): the rings as created are candidate 0; while the best so far
    // is slower than kPlacementTolerance over the expectation (the stage's
    // algorithmic bytes at the rate of the copy-third probe over the same
    // memory), up to placement_tries - 1 fresh ring sets of the same kind
    // follow, each losing set freed at once (peak: 2 ring sets + the random
    // frames).  placement_reps timed launches per candidate.
    uint32_t placement_tries = 0;
    uint32_t placement_reps = 10;
    bool placement_never_accept = false; // bench: every try runs
    // Kernel tuning (aqz_stage_bench_options; never read from the
    // environment, so a deployed library always runs the shipped kernels).
    uint32_t knobs = 0;            // A/B switches (0 = the shipped kernels)
    uint32_t nt_mode = 7;          // nontemporal policy (loads 1, L0 2, L1/2 4)
    uint32_t xcd_rot = 0;          // regions each XCD's walk is rotated by
    uint32_t region_rows_log2 = 0; // 0 = automatic
    uint64_t chunk_pad = 0;        // device bytes between chunks of a layer
    // 0 (shipped): rings of >= 256 MiB in all are packed into one arena of
    // 2 MiB virtual-memory pieces (DevBuf::kVmm), smaller ones hipMalloc'd
    // per level; otherwise (bench A/B) per-level allocations with these
    // hipExtMallocWithFlags / DevBuf flags (kRingsPlain alone = hipMalloc)
    uint32_t ring_malloc_flags = 0;
    uint64_t ring_spacer = 0;       // allocated before the rings, freed after
    uint64_t ring_arena = 0;        // > 0: every ring carved from one allocation
                                    // with this much slack (set_ring_offset)
    CodecTuning codec;             // device zstd encoder A/B switches
};

// What the creation-time placement search did (aqz_stage_placement_report).
struct PlacementReport
{
    std::vector<double> ms;       // ms per launch of every candidate
    size_t kept = 0;              // index of the kept candidate
    double kept_ms_final = 0;     // the kept placement re-timed alone
    uint64_t peak_device = 0;     // stage device bytes at the search's peak
    uint32_t reps = 0;            // timed launches per candidate
    uint32_t mode = 0;            // 3: ring arenas, 4: per-level rings
    std::vector<double> probe_gbs; // the copy-third probe over each candidate
    double probe_bus_gbs = 0;     // copy-third probe over the timing memory
    double expected_ms = 0;       // the batch's algorithmic bytes at that rate
    uint64_t alg_bytes = 0;       // algorithmic bytes of one timing launch
    bool accepted = false;        // the kept one is within the tolerance
    uint32_t stop = 0;            // 1 accepted, 2 every try ran, 3 no
                                  // expectation (probe too small), 4 OOM
};

// a candidate within this fraction over the probe's expectation ends the
// placement search
constexpr double kPlacementTolerance = 0.03;

struct LevelLayout
{
    uint64_t bytes_per_chunk;
    uint32_t chunks_per_layer;
    uint32_t layer_slots;
    uint64_t frames_per_layer;
    uint64_t frame_bytes;
    uint32_t width, height;
    uint64_t chunk_pitch;  // device bytes from chunk c to c+1 (>= bytes_per_chunk)
};

// Per-level device state shared by Stage.
struct StageLevel
{
    std::vector<Dim> dims;                 // storage order
    std::unique_ptr<ArrayDimensions> ad;   // chunk lattice of this level
    uint32_t W = 0, H = 0, planes = 0;
    bool xy_shrinks = false;               // vs previous level
    uint64_t bpc = 0;                      // bytes per chunk (the reference's)
    uint64_t pitch = 0;                    // device chunk pitch, >= bpc
    uint64_t slot_bytes = 0;               // device bytes per layer slot
    uint64_t layer_bytes = 0;              // bpc * n_chunks (host layout)
    uint32_t n_chunks = 0, n_slots = 0, F = 0;
    uint32_t tw = 0, th = 0, ntx = 0, nty = 0;
    DevBuf ring, flags, tab_off, tab_grp, ref_table;
    uint32_t period = 0;                   // n_slots * F frames
    std::vector<uint64_t> h_tab_off;
    std::vector<uint32_t> h_tab_grp;
    std::vector<int64_t> slot_layer;       // layer resident in each slot
    uint64_t frames_written = 0;           // Array::frames_written_
    uint32_t level_frame_count = 0;        // Downsampler::level_frame_count_
    DevBuf scratch;                        // row-major frames of a batch
    DevBuf partial[2];                     // carried z partial planes
    int carried = -1;                      // partial[carried] holds one
    DevBuf d_ops;
    PinnedBuf h_ops;
    hipEvent_t ops_ev = nullptr;
    // asynchronous hand-off of chunk layers (copy_layer_async): one D2H per
    // ring slot in flight; the slot's next layer waits for it
    std::vector<hipEvent_t> ready_ev, copy_ev;
    std::vector<uint8_t> copy_pending;
    // per slot: other stages' imports of the slot (import_frames), each an
    // event of the reading stage's device recorded on its stream (an event
    // is recorded only on a stream of its own device); the slot's next
    // layer waits for them
    std::vector<std::vector<std::shared_ptr<ihipEvent_t>>> peer_ev;
    DevBuf flag_bytes;                     // per slot: has_data as 0/1 bytes
    // device compression of resident layers (compress_layer): per slot the
    // frames, their offsets (device and pinned host copy) and an event
    std::unique_ptr<Compressor> comp;
    Compression comp_cfg;
    std::vector<DevBuf> cframes, coffsets;
    std::vector<PinnedBuf> h_coffsets;
    std::vector<hipEvent_t> comp_ev;
    std::vector<hipEvent_t> cdone_ev;      // the slot's frames were copied out
    std::vector<uint8_t> cdone_pending;
    std::vector<uint64_t> cdone_ticket;    // ... by this DMA-engine ticket (0: none)
    std::vector<int64_t> comp_layer;       // layer compressed in each slot
    // host-side zstd codecs (aqz_hostzstd.hh): per slot the pinned inputs
    // (shuffled or raw chunks, has_data bytes), their D2H event and the
    // host job; comp_host[slot] = the slot's compression ran on the host
    std::vector<PinnedBuf> h_zin, h_zhas;
    std::vector<hipEvent_t> zin_ev;
    std::vector<std::shared_ptr<HostLayerJob>> zjob;
    std::vector<uint8_t> comp_host;
    DevBuf d_zshuf;                        // device shuffle target
    // shard packing: compressed frames leave in shard-major order
    // (shard_index_for_chunk, then shard_internal_index); internal indices
    // of a layer = h_internal0 + (layer mod layers_per_shard) * stride
    DevBuf shard_order;
    std::vector<uint32_t> h_order, h_shard, h_internal0;
    uint32_t chunks_per_shard = 0, n_shards = 0, layers_per_shard = 1;
    uint32_t internal_stride = 0;
};

// What a stage holds (aqz_memory_usage).
struct Footprint
{
    uint64_t device = 0, pinned = 0;
};

// One chunk of a compressed layer, in output (shard-major) order.
struct ChunkEntry
{
    uint32_t chunk, shard, internal, reserved;
    uint64_t offset, nbytes;
};

// Shard::write_table_ (shard.cpp:145-166): offsets/extents as little-endian
// uint64 pairs, then the CRC-32C of those bytes.
uint32_t crc32c(const uint8_t* p, size_t n);
void shard_table(const uint64_t* offsets, const uint64_t* extents, uint32_t n,
                 uint8_t* out);

class Stage
{
  public:
    Stage(const ArrayDesc& desc, const StageOptions& opt);
    ~Stage();

    uint32_t n_levels() const { return uint32_t(lv_.size()); }
    const std::vector<Dim>& level_dims(uint32_t level) const;
    LevelLayout layout(uint32_t level) const;
    void set_stream(hipStream_t s);
    // the stage's stream waits for the work enqueued so far on s
    void wait_stream(hipStream_t s);
    void set_tuning(uint32_t knobs, uint32_t nt) { knobs_ = knobs; nt_mode_ = nt & 7u; }
    // bench: allocate fresh rings (+ has_data words, frame tables) for the
    // levels in `mask`, holding the old ones until the stage is destroyed so
    // the new ones land elsewhere (placement experiments)
    void replace_rings(uint32_t mask);
    // bench (ring_arena): move every level's ring to arena + offset (levels
    // back to back, 64 KiB aligned); the stage restarts at frame 0
    void set_ring_offset(uint64_t offset);
    void append(const void* frames, uint64_t n_frames, int mem);
    void synchronize();
    uint64_t frames_written(uint32_t level) const;
    // level-0 frames whose source bytes the stage has finished reading
    uint64_t frames_consumed();
    void wait_consumed(uint64_t frames);
    // hand-off tickets (one per copy_*_async call, 1-based, in issue order)
    uint64_t last_ticket() const { return last_ticket_; }
    uint64_t copies_completed(bool wait_all = false, uint64_t until = 0);
    void copy_layer(uint32_t level, uint64_t layer, void* dst, size_t cap,
                    uint8_t* has_data, size_t has_data_cap, int mem);
    void device_layer(uint32_t level, uint64_t layer, void** chunks,
                      uint32_t** flags);
    void copy_layer_async(uint32_t level, uint64_t layer, void* dst, size_t cap,
                          uint8_t* has_data, size_t has_data_cap);
    void wait_copies();
    // dim-1 banding: geometry and the hand-off of one complete band
    void band_geometry(uint32_t level, int32_t* supported, uint32_t* n_bands,
                       uint64_t* frames_per_band, uint32_t* chunks_per_band) const;
    void copy_band_async(uint32_t level, uint64_t layer, uint32_t band, void* dst,
                         size_t cap, uint8_t* has_data, size_t has_data_cap);
    Footprint memory_usage() const;
    // upper bound of what Stage(desc, opt) allocates (no compressed hand-off)
    static Footprint estimate_memory(const ArrayDesc& desc, const StageOptions& opt);
    // device compression of a resident layer, on the hand-off stream
    void compress_layer(uint32_t level, uint64_t layer, const Compression& c);
    // waits for that compression; offsets[0..n_chunks] (frame starts + total)
    void compressed_offsets(uint32_t level, uint64_t layer, uint64_t* offsets,
                            size_t n);
    // has that compression finished (no wait)?
    bool compression_done(uint32_t level, uint64_t layer);
    // D2H of the frames (offsets[n_chunks] bytes) on the hand-off stream
    void copy_compressed_async(uint32_t level, uint64_t layer, void* dst, size_t cap);
    // waits; one entry per chunk in output order
    void compressed_entries(uint32_t level, uint64_t layer, ChunkEntry* out, size_t n);
    void shard_geometry(uint32_t level, uint32_t* chunks_per_shard, uint32_t* n_shards,
                        uint32_t* layers_per_shard) const;
    void finalize();
    // the level-0 tile split on the host (level0_on_host; aqz_hostsplit.hh):
    // frames [first, first + n) over the stage's host threads, or rows of
    // one frame on the calling thread, into the packed chunks [chunk0,
    // chunk0 + cap / bytes_per_chunk) of a layer
    void split_level0_host(const void* frames, uint64_t n, uint64_t first, uint32_t chunk0,
                           void* dst, size_t cap, uint8_t* has_data, size_t has_data_cap);
    void split_level0_rows(const void* frame, uint64_t frame_id, uint32_t row_begin,
                           uint32_t row_end, void* frame_copy, uint32_t chunk0, void* dst,
                           size_t cap, uint8_t* has_data, size_t has_data_cap) const;
    // z-slab assembly: frames [first, first + count) of `layer` of `level`
    // (layer-local frame ids) copied from src's resident layer -- or zeroed
    // when src is null -- with their has_data, after the work enqueued so far
    // on src; src's slot is not rewritten until the copy has run
    void import_frames(Stage* src, uint32_t level, uint64_t layer, uint32_t first,
                       uint32_t count);
    int device() const { return desc_.device; }
    void enable_timing(bool on);
    void timing(double* total_ms, uint64_t* launches);
    // timing events on the stage's stream bracketing a region of appends
    void mark(int which);
    double marked_ms();
    const char* dominant_kernel() const;
    uint32_t zstd_far_ranges(uint32_t level) const
    {
        if (level >= lv_.size())
            throw Error(3, "level out of range");
        return lv_[level].comp ? lv_[level].comp->far_ranges() : 0;
    }
    int numa_node() const { return numa_node_; }
    size_t numa_cpus() const { return numa_cpus_.size(); }
    // pin the calling thread to the CPUs of the device's NUMA node
    void bind_host_thread() const { pin_current_thread(numa_cpus_); }
    // placement calibration: ms per candidate launch and the one kept
    const std::vector<double>& placement_ms() const { return placement_.ms; }
    size_t placement_best() const { return placement_.kept; }
    const PlacementReport& placement() const { return placement_; }

  private:
    struct Pending
    {
        bool has = false;
        int kind = 0; // 0: level k-1 frame in batch, 1: carried partial
        uint32_t index = 0;
        bool scale = false;
    };

    void run_batch(const uint8_t* dsrc, uint32_t n);
    void place_level(StageLevel& L, uint8_t* at = nullptr);
    void place_rings_at(uint64_t offset);
    void calibrate_placement();
    void build_shard_order(StageLevel& L);
    void ensure_comp_slots(StageLevel& L);
    void compress_layer_host(StageLevel& L, uint32_t slot, uint64_t layer,
                             const Compression& c);
    FusedParams fused_params(const uint8_t* dsrc, uint32_t n, uint32_t n_fused,
                             uint32_t rh_log2, bool tail);
    void run_fused(const uint8_t* dsrc, uint32_t n);
    void run_fused3d(const uint8_t* dsrc, uint32_t n);
    void run_generic(const uint8_t* dsrc, uint32_t n);
    void enter_layers(StageLevel& L, uint64_t first_fid, uint64_t n);
    void enter_layer(StageLevel& L, uint64_t layer);
    LevelGeom geom(StageLevel& L, uint64_t fid0, bool tiles,
                   uint8_t* scratch) const;
    void tile_addr(const StageLevel& L, uint64_t fid, uint64_t* off,
                   uint32_t* flag_off, uint32_t* tag) const;
    const uint8_t* frame_ptr(uint32_t level, uint32_t index,
                             const uint8_t* dsrc) const;

    ArrayDesc desc_;
    StageOptions opt_;
    size_t bpp_;
    std::vector<StageLevel> lv_;
    bool fused_2d_ = true;
    bool fused_3d_ = false;  // regular 2x2x2 schedule: fused_pyramid_3d
    uint32_t g3d_ = 1, zmask3d_ = 0;
    uint32_t n_fused_ = 0;
    uint32_t rh_log2_ = 4;
    uint64_t max_frames_ = 0; // 0 = unbounded
    // z-slab schedule: level-0 frames per slab, frames of the current slab
    // written, and every level's frame-id jump at the end of a slab
    uint64_t slab_len_ = 0, slab_done_ = 0;
    std::vector<uint64_t> slab_skip_;
    hipStream_t own_stream_ = nullptr;
    hipStream_t stream_ = nullptr;
    // host-source staging: pinned double buffer -> device double buffer.
    // H2D runs on h2d_ (batch i+1's copy overlaps batch i's kernels), layer
    // hand-off D2H on d2h_; events order them against stream_.
    PinnedBuf h_stage_[2];
    DevBuf d_stage_[2];
    hipEvent_t h2d_ev_[2] = { nullptr, nullptr };     // H2D of buffer j done
    hipEvent_t consume_ev_[2] = { nullptr, nullptr }; // kernels read buffer j
    bool consume_rec_[2] = { false, false };
    int stage_idx_ = 0;
    hipStream_t h2d_ = nullptr, d2h_ = nullptr;
    // device compression of handed-off layers runs on comp_, so layer i+1
    // compresses while layer i's frames go D2H on d2h_
    hipStream_t comp_ = nullptr;
    hipStream_t comp_lo_ = nullptr;  // compression of levels 1-2
    hipStream_t comp_lo2_ = nullptr; // levels >= 3 (least priority: a queue pool of its own)
    hipStream_t comp_stream(const StageLevel& L) const
    {
        const size_t k = size_t(&L - &lv_[0]);
        return k == 0 ? comp_ : k <= 2 ? comp_lo_ : comp_lo2_;
    }
    std::unique_ptr<CopyPool> pool_;
    std::unique_ptr<TaskPool> zpool_; // host zstd workers
    std::unique_ptr<SplitPool> split_pool_; // host level-0 split workers
    // CPUs of the device's NUMA node: the host pools run there (AQZ_NUMA=0
    // turns it off)
    std::vector<int> numa_cpus_;
    int numa_node_ = -1;
    // XY-transposed storage order: level-0 frames are transposed into xbuf_
    // (acquisition rows x cols -> storage rows x cols) before the pipeline
    bool xy_ = false;
    bool xy_direct_ = false; // XY transpose fused into the strip kernel's loads
    bool xy_src_ = false;    // the batch being launched is in acquisition order
    uint32_t acq_rows_ = 0, acq_cols_ = 0;
    DevBuf xbuf_;
    // source consumption: (event, appended frames when it fires)
    std::vector<std::pair<hipEvent_t, uint64_t>> inflight_;
    size_t inflight_head_ = 0;
    std::vector<hipEvent_t> free_ev_;
    uint64_t appended_ = 0, consumed_ = 0;
    // a hand-off copy not yet retired: a HIP event on d2h_, or the signal
    // of a copy on a DMA engine (sdma_d2h_)
    struct Ticket
    {
        hipEvent_t ev = nullptr;
        hsa_signal_t sig{ 0 };
    };
    std::deque<Ticket> tickets_;
    uint64_t tickets_issued_ = 0, tickets_done_ = 0, last_ticket_ = 0;
    uint64_t issue_ticket();
    uint64_t issue_ticket(hsa_signal_t sig);
    // compressed frames D2H on an SDMA engine (hsa_amd_memory_async_copy)
    // instead of HIP's blit kernels (AQZ_D2H_SDMA=1, A/B)
    bool sdma_d2h_ = false;
    hsa_agent_t hsa_gpu_{ 0 }, hsa_cpu_{ 0 };
    std::vector<hsa_signal_t> free_sig_;
    void note_consumed(hipStream_t s, uint64_t frames);
    void retire_consumed(bool wait);
    uint32_t nt_mode_ = 7;           // nontemporal policy: input loads (1), level-0 (2) and level-1/2 (4) stores
    uint32_t knobs_ = 0;             // tuning A/B switches
    uint32_t xcd_rot_ = 0;           // regions each XCD's walk is rotated by, per XCD index
    std::vector<Pending> pend_;
    // kernel timing
    bool timing_ = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pairs_;
    size_t ev_used_ = 0;
    double timed_ms_ = 0;
    uint64_t timed_launches_ = 0;
    hipEvent_t mark_ev_[2] = { nullptr, nullptr };
    hipEvent_t ext_ev_ = nullptr;  // wait_stream
    PlacementReport placement_;         // creation-time placement search
    std::vector<DevBuf> held_;          // replace_rings: old rings kept allocated
    DevBuf arena_;                      // every level's ring (the shipped arena)
    uint64_t arena_rings_ = 0;          // bytes of the rings inside it
    bool arena_fallback_ = false;       // the VMM arena failed: per-level rings
    std::mutex access_mu_;              // grant_access, StageLevel::peer_ev
    std::vector<int> granted_;          // devices mapped into a VMM arena
    // import_frames from another device reads this stage's rings: a
    // virtual-memory arena must be mapped for that device too
    void grant_access(int device);
    bool finalized_ = false;
};

// Downsampler::downsampling_method / get_metadata().dump() (downsampler.cpp:
// 422-485) for a method value; throw Error(1) on an invalid method.
const char* downsampling_method_name(int32_t method);
std::string downsampling_metadata_json(int32_t method);

class GpuDownsampler
{
  public:
    explicit GpuDownsampler(const ArrayDesc& desc);
    ~GpuDownsampler();

    uint32_t n_levels() const { return uint32_t(levels_.size()); }
    const std::vector<Dim>& level_dims(uint32_t level) const;
    void add_frame(const void* frame, size_t nbytes, int mem);
    bool take_frame(uint32_t level, void* dst, size_t cap, int mem,
                    size_t* nbytes);
    const char* method_name() const;
    std::string metadata_json() const;

  private:
    struct Lv
    {
        uint32_t W, H, planes;
        bool xy_shrinks;
        DevBuf cur, pending, partial;
        bool has_pending = false, has_partial = false;
        uint32_t count = 0;
    };
    int32_t dtype_, method_;
    size_t bpp_;
    std::vector<std::vector<Dim>> levels_;
    std::vector<Lv> lv_;
    DevBuf input_;
    DevBuf d_op_;
    hipStream_t stream_ = nullptr;
    int32_t device_;
};

} // namespace aqz
