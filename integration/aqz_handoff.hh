// aqz_handoff.hh -- the consumer-thread side of the MI355X stage for one
// multiscale array, independent of zarr::Array so that it runs (and is
// tested, tests/native/handoff_replay.cpp) without the reference library.
//
// It replaces, for a multiscale array, what the reference's consumer thread
// does per frame (MultiscaleArray::write_frame, multiscale.array.cpp:57-74,
// 291-325, and Array::write_frame, array.cpp:153-223) and what its flush
// jobs do per chunk (Array::dispatch_chunk_job_, array.cpp:664-760):
//
//   * frames are copied into one of two pinned batch buffers (by a few copy
//     threads); a full batch is appended asynchronously (aqz_stage_append
//     reads pinned memory by DMA) and the buffer is refilled only after
//     aqz_stage_wait_consumed says the stage has read it -- the frame
//     queue's buffer swap (frame.queue.cpp:48-73) without a spin;
//   * every unit of every level is handed off as soon as its frames are
//     written: a dim-1 band where Array::flush_completed_bands_ applies
//     (array.cpp:873-908), else a chunk layer (should_flush_, array.cpp:
//     910-922).  Raw units are copied D2H (aqz_stage_copy_band_async /
//     aqz_stage_copy_layer_async); with a codec the whole layer is
//     compressed on the device (aqz_stage_compress_layer, the codecs of
//     Chunk::compress_and_take_buffer, chunk.cpp:78-106) and only its frames
//     cross PCIe, once the compression has finished (aqz_stage_compression_
//     done) -- the consumer thread never waits for a kernel;
//   * a unit whose copy has landed (hand-off tickets complete in issue
//     order) goes to the sink strictly in frame order per level, with a
//     Lease on its host buffer: the sink's writer jobs hold the lease, and
//     the buffer is refilled only once every lease is released.
//
// Device selection (no ABI change): select_device() reads
// AQZ_DEVICE.
#pragma once

#include "aqz_gpu.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace aqz_binding {

// A reference on a host hand-off buffer.  The Handoff refills a buffer only
// when no lease on it is alive; a sink copies the lease into every job that
// reads the buffer after unit() returned.
class Lease
{
  public:
    Lease() = default;
    explicit Lease(std::atomic<int>* pins)
      : p_(pins)
    {
        if (p_)
            p_->fetch_add(1);
    }
    Lease(const Lease& o)
      : Lease(o.p_)
    {
    }
    Lease(Lease&& o) noexcept
      : p_(o.p_)
    {
        o.p_ = nullptr;
    }
    Lease& operator=(Lease o) noexcept
    {
        std::swap(p_, o.p_);
        return *this;
    }
    ~Lease() { release(); }
    void release()
    {
        if (p_ && p_->fetch_sub(1) == 1)
            p_->notify_all();
        p_ = nullptr;
    }

  private:
    std::atomic<int>* p_ = nullptr;
};

// One handed-off unit of a level: chunk slots [c0, c0 + n_chunks) of a chunk
// layer, raw (chunks + has_data) or compressed (frames + entries, the whole
// layer in shard-major order).
struct Unit
{
    uint32_t level = 0;
    uint64_t layer = 0;   // chunk layer of the level (frames_written / F)
    uint32_t band = 0, n_bands = 1;
    uint32_t c0 = 0, n_chunks = 0;
    uint64_t first = 0;   // the unit's first frame id of the level
    uint64_t frames = 0;  // frames of the level inside this unit
    bool complete = true; // false only at close: the zero-filled remainder
    bool last_in_layer = true;
    uint64_t bytes_per_chunk = 0;
    // raw
    const uint8_t* chunks = nullptr;   // n_chunks x bytes_per_chunk
    const uint8_t* has_data = nullptr; // n_chunks bytes
    // compressed
    const uint8_t* data = nullptr;     // the layer's frames back to back
    const aqz_chunk_entry* entries = nullptr; // n_chunks, shard-major
    Lease lease;
};

struct HandoffSink
{
    virtual ~HandoffSink() = default;
    // units arrive in frame order per level; non-success stops the stream
    virtual aqz_status unit(Unit& u) = 0;
};

// ---- shard routing of a level's units ---------------------------------------
// What a level's zarr::Array does with a completed unit's chunks and frames,
// independent of the reference library so that the binding (GpuArray,
// integration/multiscale.array.gpu.cpp) and the GPU replay
// (tests/native/handoff_replay.cpp) run the same routing code.

// The index math the router needs (ArrayDimensions, array.dimensions.cpp:
// 376-548): the reference's own in the binding, aqz_dims in the replay.
struct ShardMap
{
    virtual ~ShardMap() = default;
    virtual uint32_t chunks_in_memory() const = 0; // number_of_chunks_in_memory
    virtual uint32_t number_of_shards() const = 0;
    virtual uint32_t shard_index_for_chunk(uint32_t chunk) const = 0;
    virtual uint32_t shard_internal_index(uint32_t chunk) const = 0;
    virtual std::vector<uint32_t> skipped_internal_indices(uint32_t shard,
                                                           uint32_t layer) const = 0;
};

// What the router asks of the array it routes for: the Shard::write_chunk /
// skip_chunk jobs on the thread pool (Array::dispatch_chunk_job_ /
// dispatch_skip_job_, array.cpp:624-760), should_rollover_ (array.cpp:
// 924-937, asked after the unit's frames are counted) and rollover_ with
// write_metadata_ (array.cpp:939-951, 213-216).
struct ShardWriter
{
    static constexpr uint32_t kPadding = 0xffffffffu; // skip_chunk of ragged padding
    virtual ~ShardWriter() = default;
    // chunk: the chunk index (current layer * chunks in memory + slot)
    virtual void write_chunk(uint32_t shard, uint32_t internal, uint32_t chunk,
                             const uint8_t* bytes, size_t n, const Lease& lease) = 0;
    // chunk: as above for a chunk without data, kPadding for ragged padding
    virtual void skip_chunk(uint32_t shard, uint32_t internal, uint32_t chunk) = 0;
    virtual bool should_rollover() = 0;
    virtual void rollover() = 0;
};

class ShardRouter
{
  public:
    explicit ShardRouter(const ShardMap& map)
      : map_(map)
    {
    }

    // The chunk layer inside the current append-dimension shard row
    // (Array::current_layer_).
    uint32_t current_layer() const { return current_layer_; }

    // Every chunk of the unit to its shard: chunk index = current_layer *
    // chunks_in_memory + the chunk's slot in the layer (compress_and_flush_
    // data_ / compress_and_flush_band_, array.cpp:762-871); bytes go to
    // write_chunk, a chunk without data to skip_chunk (the job's has_data
    // test, array.cpp:713-720).  On a layer's last unit the ragged padding
    // of every shard is skipped so each shard's countdown completes
    // (array.cpp:771-790, 852-862).  A compressed unit's entries carry the
    // device's (shard, internal) of each chunk: they must all agree with the
    // map -- checked before any chunk is dispatched -- else INTERNAL_ERROR
    // and nothing of the unit is routed.
    aqz_status route(const Unit& u, ShardWriter& w) const
    {
        const uint32_t n_mem = map_.chunks_in_memory();
        const uint32_t offset = current_layer_ * n_mem;
        for (uint32_t i = 0; i < u.n_chunks; ++i) {
            const uint32_t local = u.entries ? u.entries[i].chunk : u.c0 + i;
            if (local >= n_mem)
                return AQZ_STATUS_INTERNAL_ERROR;
            if (u.entries && (u.entries[i].shard != map_.shard_index_for_chunk(offset + local) ||
                              u.entries[i].internal != map_.shard_internal_index(offset + local)))
                return AQZ_STATUS_INTERNAL_ERROR;
        }
        for (uint32_t i = 0; i < u.n_chunks; ++i) {
            uint32_t local;
            const uint8_t* p;
            size_t n;
            if (u.entries) {
                const aqz_chunk_entry& e = u.entries[i];
                local = e.chunk;
                p = u.data + e.offset;
                n = e.nbytes;
            } else {
                local = u.c0 + i;
                p = u.chunks + size_t(i) * u.bytes_per_chunk;
                n = u.has_data[i] ? u.bytes_per_chunk : 0;
            }
            const uint32_t chunk = offset + local;
            const uint32_t shard = map_.shard_index_for_chunk(chunk);
            const uint32_t internal = map_.shard_internal_index(chunk);
            if (n == 0)
                w.skip_chunk(shard, internal, chunk);
            else
                w.write_chunk(shard, internal, chunk, p, n, u.lease);
        }
        if (u.last_in_layer)
            for (uint32_t s = 0; s < map_.number_of_shards(); ++s)
                for (const uint32_t idx : map_.skipped_internal_indices(s, current_layer_))
                    w.skip_chunk(s, idx, ShardWriter::kPadding);
        return AQZ_STATUS_SUCCESS;
    }

    // After the unit's frames were counted: a layer's last complete unit
    // ends the layer -- rollover to a new append-dimension shard row when
    // should_rollover_ says so, else the next layer (Array::write_frame's
    // tail, array.cpp:209-219; compress_and_flush_data_, :799-803;
    // flush_completed_bands_, :880-898).  The last, partial layer at close
    // (complete = false) ends nothing.  Returns true on a rollover.
    bool commit(const Unit& u, ShardWriter& w)
    {
        if (!(u.last_in_layer && u.complete))
            return false;
        if (w.should_rollover()) {
            w.rollover();
            current_layer_ = 0;
            return true;
        }
        ++current_layer_;
        return false;
    }

  private:
    const ShardMap& map_;
    uint32_t current_layer_ = 0;
};

// The per-array counters zarr::Array keeps frame by frame (the tail of
// Array::write_frame, array.cpp:196-219; flush_completed_bands_, :873-908),
// advanced a whole unit of frames at a time.  GpuArray mirrors them into
// the reference's members (frames_written_() = total_bytes_written_ /
// bytes_per_frame_ is what should_rollover_ reads, array.cpp:924-937,
// 974-977); the GPU replay runs the same code and checks it, unit by unit,
// against the reference's per-frame rules.
struct ArrayLedger
{
    uint64_t total_bytes_written = 0;
    uint64_t last_successful_frame_id = 0;
    // bytes of frames not yet handed to their shards: 0 after every unit
    // (the reference zeroes it at each layer flush; its only reader,
    // Array::close_, array.cpp:380-383, must find nothing left to flush)
    uint64_t bytes_to_flush = 0;
    uint32_t flushed_band_count = 0; // bands of the current layer flushed

    uint64_t frames_written(uint64_t bytes_per_frame) const
    {
        return bytes_per_frame ? total_bytes_written / bytes_per_frame : 0;
    }

    // The unit's frames are written: false (nothing changes) when they would
    // pass max_bytes (Array::write_frame's bounds check, array.cpp:174-177;
    // 0 = unbounded).
    bool commit(const Unit& u, uint64_t bytes_per_frame, uint64_t max_bytes)
    {
        const uint64_t nbytes = u.frames * bytes_per_frame;
        if (max_bytes > 0 && total_bytes_written + nbytes > max_bytes)
            return false;
        if (u.frames)
            last_successful_frame_id = frames_written(bytes_per_frame) + u.frames - 1;
        total_bytes_written += nbytes;
        bytes_to_flush = 0;
        // a layer's last band resets the count (array.cpp:884-896), an
        // interior band leaves band + 1 flushed (:897-905)
        flushed_band_count = u.last_in_layer ? 0 : u.band + 1;
        return true;
    }
};

// aqz_dims as the router's ShardMap (the replay; any caller without the
// reference's ArrayDimensions).  Does not own d.
class DimsShardMap final : public ShardMap
{
  public:
    explicit DimsShardMap(const aqz_dims* d)
      : d_(d)
    {
        (void)aqz_dims_shard_geometry(d_, nullptr, &n_shards_, &layers_per_shard_);
    }
    uint32_t chunks_in_memory() const override
    {
        return aqz_dims_number_of_chunks_in_memory(d_);
    }
    uint32_t number_of_shards() const override { return n_shards_; }
    uint32_t layers_per_shard() const { return layers_per_shard_; }
    uint32_t shard_index_for_chunk(uint32_t c) const override
    {
        return aqz_dims_shard_index_for_chunk(d_, c);
    }
    uint32_t shard_internal_index(uint32_t c) const override
    {
        return aqz_dims_shard_internal_index(d_, c);
    }
    std::vector<uint32_t> skipped_internal_indices(uint32_t shard,
                                                   uint32_t layer) const override
    {
        size_t n = 0;
        if (aqz_dims_skipped_internal_indices(d_, shard, layer, nullptr, 0, &n) !=
              AQZ_STATUS_SUCCESS ||
            n == 0)
            return {};
        std::vector<uint32_t> v(n);
        (void)aqz_dims_skipped_internal_indices(d_, shard, layer, v.data(), n, &n);
        return v;
    }

  private:
    const aqz_dims* d_;
    uint32_t n_shards_ = 1, layers_per_shard_ = 1;
};

struct HandoffOptions
{
    uint32_t batch_frames = 64; // frames per append
    uint32_t host_slots = 3;    // host unit buffers per level (>= 1)
    uint32_t copy_threads = 8;  // threads copying frames into the batch
    aqz_compression comp{};     // codec 0: raw chunk units
    // Raw units only: level 0 is tile-split on the host by the copy threads
    // in the same pass that copies each frame into the pinned batch (the
    // stages are created with aqz_stage_options.level0_split_on_host): only
    // levels >= 1 cross PCIe back.
    bool level0_on_host = false;
};

// Whether an array takes the host split of level 0 (HandoffOptions::
// level0_on_host, aqz_stage_options.level0_split_on_host): a raw hand-off
// of an array whose storage rows are its acquisition rows.
inline bool
level0_on_host_for(const aqz_array_desc& desc, const aqz_compression& comp)
{
    const size_t nd = desc.dimension_count;
    const bool xy = desc.storage_dimension_order && nd >= 2 &&
                    desc.storage_dimension_order[nd - 1] != nd - 1;
    return comp.codec == AQZ_CODEC_NONE && !xy;
}

// AQZ_DEVICE (a deployment setting read where the reference configures an
// array, zarr.stream.cpp:1231-1279; no ABI change):
//   unset or "auto"  the next device, round robin over the visible devices,
//                    per multiscale array created by the process (BASELINE
//                    configs[4]: one camera stream per GPU);
//   "N"              device N;  "a,b,..." round robin over that list;
//   "off" or "-1"    no GPU: the reference's CPU path.
// Returns -1 for "no GPU".
inline int32_t
select_device(int32_t n_visible)
{
    static std::atomic<uint32_t> next{ 0 };
    const char* e = std::getenv("AQZ_DEVICE");
    std::string s = e ? e : "auto";
    if (s == "off" || s == "-1" || n_visible <= 0)
        return -1;
    std::vector<int32_t> list;
    if (s == "auto" || s.empty()) {
        for (int32_t d = 0; d < n_visible; ++d)
            list.push_back(d);
    } else {
        size_t i = 0;
        while (i < s.size()) {
            const size_t j = std::min(s.find(',', i), s.size());
            const int32_t d = std::atoi(s.substr(i, j - i).c_str());
            if (d < 0 || d >= n_visible)
                return -1;
            list.push_back(d);
            i = j + 1;
        }
        if (list.empty())
            return -1;
    }
    return list[next.fetch_add(1) % list.size()];
}

// z slabs of a volume stream over several stages (BASELINE
// configs[3]): level-0 planes [begin, end) of every z stack go to stage r.
// The bounds are multiples of 2^(z-halving levels), so no z pair straddles
// two stages (aqz_stage_options.z_slab_*).
struct SlabPlan
{
    uint32_t planes = 0;                // level-0 z planes per stack (0: one stage)
    std::vector<uint32_t> begin, end;   // level-0 slab of each stage
};

// AQZ_Z_SLABS = N: a multiscale array whose dimension before y is a z
// (Space) dimension is split into N z slabs, one stage (GPU) each.  Returns
// the plan (empty when N < 2 or the z extent cannot be split evenly
// enough: every slab at least `align` planes).
inline SlabPlan
plan_z_slabs(uint32_t planes, uint32_t n, uint32_t align)
{
    SlabPlan p;
    align = std::max<uint32_t>(1, align);
    if (n < 2 || planes == 0 || planes % align != 0 || planes / align < n)
        return p;
    const uint32_t units = planes / align;
    p.planes = planes;
    for (uint32_t r = 0; r < n; ++r) {
        p.begin.push_back(uint32_t(uint64_t(units) * r / n) * align);
        p.end.push_back(uint32_t(uint64_t(units) * (r + 1) / n) * align);
    }
    return p;
}

inline uint32_t
slabs_from_env()
{
    const char* e = std::getenv("AQZ_Z_SLABS");
    const int n = e ? std::atoi(e) : 1;
    return n > 1 ? uint32_t(n) : 1u;
}

// The drop-in's own memory for one multiscale array on the GPU path, beyond
// what ZarrStreamSettings_estimate_max_memory_usage counts for it
// (acquire.zarr.cpp:216-314: the frame queue and the array's frame buffer
// stay the reference's).  An upper bound, with no GPU needed:
//   host   -- the hand-off's pinned buffers (Handoff::host_bytes: a batch
//             double buffer per stage, host_slots unit buffers per level at
//             the codec's capacity with their has_data bytes), every
//             stage's pinned memory (aqz_stage_estimate_memory) and, per
//             compressed level and ring slot, the read-back of the frame
//             offsets (and with AQZ_ZSTD_HOST the shuffled layer);
//   device -- every stage's aqz_stage_estimate_memory (creation-time
//             placement peak included), and per compressed level and ring
//             slot the frames (aqz_compressor_max_bytes) and offsets, plus
//             the codec's scratch (aqz_compressor_scratch_bytes).
struct MemoryEstimate
{
    uint64_t host_bytes = 0, device_bytes = 0;
};

inline aqz_status
estimate_memory(const aqz_array_desc& desc, const aqz_stage_options& opt,
                const HandoffOptions& o, uint32_t n_stages, MemoryEstimate* out)
{
    if (!out || n_stages == 0)
        return AQZ_STATUS_INVALID_ARGUMENT;
    *out = MemoryEstimate{};
    aqz_memory_usage st{};
    aqz_status s = aqz_stage_estimate_memory(&desc, &opt, &st);
    if (s != AQZ_STATUS_SUCCESS)
        return s;
    // the levels' storage-order dims, as the stage makes them
    aqz_dims* base = nullptr;
    s = aqz_dims_create(desc.dimensions, desc.dimension_count, desc.data_type,
                        desc.storage_dimension_order, &base);
    if (s != AQZ_STATUS_SUCCESS)
        return s;
    std::vector<aqz_dimension> d0(aqz_dims_ndims(base));
    for (size_t i = 0; i < d0.size(); ++i)
        (void)aqz_dims_get(base, i, &d0[i]);
    aqz_dims_destroy(base);
    uint32_t nl = 0;
    s = aqz_pyramid_levels(d0.data(), d0.size(), desc.max_levels, &nl, nullptr, 0);
    std::vector<aqz_dimension> lv(size_t(nl) * d0.size());
    if (s == AQZ_STATUS_SUCCESS)
        s = aqz_pyramid_levels(d0.data(), d0.size(), desc.max_levels, &nl, lv.data(),
                               lv.size());
    if (s != AQZ_STATUS_SUCCESS)
        return s;
    const size_t nd = d0.size();
    static const size_t bpp_of[] = { 1, 2, 4, 8, 1, 2, 4, 8, 4, 8 };
    const size_t bpp = desc.data_type >= 0 && desc.data_type < 10 ? bpp_of[desc.data_type] : 8;
    const uint64_t fb = uint64_t(d0[nd - 1].array_size_px) * d0[nd - 2].array_size_px * bpp;
    const uint32_t batch = std::max<uint32_t>(1, o.batch_frames);
    const uint32_t B = opt.max_batch_frames ? opt.max_batch_frames : 64;
    const uint32_t slots = std::max<uint32_t>(1, o.host_slots);
    const bool compressed = o.comp.codec != AQZ_CODEC_NONE;
    const char* hz = std::getenv("AQZ_ZSTD_HOST");
    const bool host_zstd = hz && std::atoi(hz) != 0 &&
                           (o.comp.codec == AQZ_CODEC_BLOSC_ZSTD || o.comp.codec == AQZ_CODEC_ZSTD);
    uint64_t host = uint64_t(n_stages) * (2 * uint64_t(batch) * fb + st.pinned_bytes);
    uint64_t dev = uint64_t(n_stages) * st.device_bytes;
    for (uint32_t l = 0; l < nl; ++l) {
        aqz_dims* d = nullptr;
        s = aqz_dims_create(&lv[size_t(l) * nd], nd, desc.data_type, nullptr, &d);
        if (s != AQZ_STATUS_SUCCESS)
            return s;
        const uint64_t bpc = aqz_dims_bytes_per_chunk(d);
        const uint32_t n_chunks = aqz_dims_number_of_chunks_in_memory(d);
        const uint64_t F = std::max<uint64_t>(1, aqz_dims_frames_per_chunk_layer(d));
        int32_t banded = 0;
        uint32_t n_bands = 1, per_band = n_chunks;
        uint64_t fpb = 0;
        (void)aqz_dims_dim1_banding(d, &banded, &n_bands, &fpb, &per_band);
        aqz_dims_destroy(d);
        if (compressed || !banded)
            per_band = n_chunks;
        const uint64_t cap =
          compressed ? aqz_compressor_max_bytes(bpc, n_chunks) : bpc * per_band;
        host += uint64_t(slots) * (cap + per_band);
        if (!compressed)
            continue;
        const uint64_t ring_slots =
          std::max<uint64_t>(opt.layer_slots ? opt.layer_slots : 2, (B - 1 + F - 1) / F + 1);
        const uint64_t offs = (uint64_t(n_chunks) + 1) * 8;
        uint64_t ldev = ring_slots * (aqz_compressor_max_bytes(bpc, n_chunks) + offs) +
                        aqz_compressor_scratch_bytes(&o.comp, bpc, uint32_t(bpp), n_chunks);
        uint64_t lhost = ring_slots * offs;
        if (host_zstd) {
            ldev += bpc * n_chunks; // the shuffled layer
            lhost += ring_slots * (bpc * n_chunks + n_chunks);
        }
        dev += uint64_t(n_stages) * ldev;
        host += uint64_t(n_stages) * lhost;
    }
    out->host_bytes = host;
    out->device_bytes = dev;
    return AQZ_STATUS_SUCCESS;
}

class Handoff
{
  public:
    // One stage: the whole stream.  Several stages: stage r receives z
    // slab r of every stack (created with aqz_stage_options.z_slab_begin /
    // z_slab_end = plan.begin[r] / plan.end[r]); every unit is assembled in
    // one of them (aqz_stage_import_frames, over xGMI) and handed off from
    // there.
    Handoff(std::vector<aqz_stage*> stages, const SlabPlan& plan, uint64_t frame_bytes,
            const HandoffOptions& o, HandoffSink& sink)
      : st_(std::move(stages))
      , plan_(plan)
      , frame_bytes_(frame_bytes)
      , opt_(o)
      , sink_(sink)
    {
        opt_.batch_frames = std::max<uint32_t>(1, opt_.batch_frames);
        opt_.host_slots = std::max<uint32_t>(1, opt_.host_slots);
        if (st_.empty() || (st_.size() > 1 && plan_.begin.size() != st_.size())) {
            status_ = AQZ_STATUS_INVALID_ARGUMENT;
            return;
        }
        in_.resize(st_.size());
        for (Input& in : in_)
            for (int j = 0; j < 2; ++j)
                status_ =
                  worse(status_, aqz_host_alloc(size_t(opt_.batch_frames) * frame_bytes_,
                                                reinterpret_cast<void**>(&in.buf[j])));
        aqz_stage* st0 = st_[0];
        const uint32_t nl = aqz_stage_n_levels(st0);
        levels_.resize(nl);
        for (uint32_t l = 0; l < nl && status_ == AQZ_STATUS_SUCCESS; ++l) {
            Level& L = levels_[l];
            status_ = worse(status_, aqz_stage_level_layout(st0, l, &L.lay));
            int32_t banded = 0;
            status_ = worse(status_, aqz_stage_band_geometry(st0, l, &banded, &L.n_bands,
                                                             &L.frames_per_band,
                                                             &L.chunks_per_band));
            // a compressed unit is a whole layer (the device compresses
            // layers); raw units follow the reference's dim-1 bands
            L.compressed = opt_.comp.codec != AQZ_CODEC_NONE;
            L.host = l == 0 && opt_.level0_on_host;
            if (L.host && L.compressed)
                status_ = worse(status_, AQZ_STATUS_INVALID_ARGUMENT);
            if (L.compressed || !banded) {
                L.n_bands = 1;
                L.frames_per_band = L.lay.frames_per_layer;
                L.chunks_per_band = L.lay.chunks_per_layer;
            }
            if (st_.size() > 1) {
                // z planes of this level (the dimension before y)
                aqz_dimension d[16];
                size_t nd = 0;
                status_ = worse(status_, aqz_stage_level_dims(st0, l, d, 16, &nd));
                L.planes = nd >= 3 ? d[nd - 3].array_size_px : 0;
                if (L.planes == 0 || plan_.planes % L.planes != 0)
                    status_ = worse(status_, AQZ_STATUS_INVALID_SETTINGS);
            }
            const size_t cap =
              L.compressed ? size_t(aqz_compressor_max_bytes(L.lay.bytes_per_chunk,
                                                            L.lay.chunks_per_layer))
                           : size_t(L.lay.bytes_per_chunk) * L.chunks_per_band;
            for (uint32_t i = 0; i < opt_.host_slots; ++i) {
                auto s = std::make_unique<Slot>();
                s->cap = cap;
                status_ = worse(status_, aqz_host_alloc(cap, reinterpret_cast<void**>(&s->buf)));
                status_ = worse(status_, aqz_host_alloc(L.chunks_per_band,
                                                        reinterpret_cast<void**>(&s->has)));
                // the host split never writes ragged padding (chunk.cpp:8-15):
                // it must start zero
                if (L.host && s->buf)
                    std::memset(s->buf, 0, cap);
                s->ent.resize(L.chunks_per_band);
                L.slots.push_back(std::move(s));
            }
            if (L.host) {
                // a ragged last dim-1 band leaves internal positions that
                // the other bands fill: its slot is cleared when a full
                // band used it last
                L.ragged_last_band =
                  L.n_bands > 1 &&
                  L.lay.frames_per_layer - uint64_t(L.n_bands - 1) * L.frames_per_band <
                    L.frames_per_band;
                rows_ = L.lay.height;
                row_bytes_ = L.lay.height ? L.lay.frame_bytes / L.lay.height : 0;
            }
        }
        const uint32_t nt = std::max<uint32_t>(1, opt_.copy_threads);
        for (uint32_t t = 1; t < nt; ++t)
            copiers_.emplace_back([this, t] {
                (void)aqz_stage_bind_host_thread(st_[0]); // next to the device
                copier_(t);
            });
    }

    Handoff(aqz_stage* st, uint64_t frame_bytes, const HandoffOptions& o, HandoffSink& sink)
      : Handoff(std::vector<aqz_stage*>{ st }, SlabPlan{}, frame_bytes, o, sink)
    {
    }

    ~Handoff()
    {
        {
            std::lock_guard<std::mutex> lk(cmu_);
            cstop_ = true;
        }
        ccv_.notify_all();
        for (auto& t : copiers_)
            t.join();
        // units still in flight must land, and every lease end, before the
        // buffers are freed
        for (aqz_stage* s : st_)
            (void)aqz_stage_wait_copies(s);
        for (Level& L : levels_)
            for (auto& s : L.slots) {
                wait_pins_(*s);
                aqz_host_free(s->buf);
                aqz_host_free(s->has);
            }
        for (Input& in : in_)
            for (uint8_t* b : in.buf)
                aqz_host_free(b);
    }

    Handoff(const Handoff&) = delete;
    Handoff& operator=(const Handoff&) = delete;

    aqz_status status() const { return status_; }
    uint64_t frames_accepted() const { return accepted_; }

    // Where the consumer thread's time went, in nanoseconds (for a caller
    // that traces the hand-off; tests/native/handoff_replay prints it):
    // write_frame in all, and inside it the wait for a batch buffer the stage
    // has not read yet, the frame copy (+ level-0 split), the waits for a free
    // host unit buffer and the appends.  sink: the units handed to the sink
    // (HandoffSink::unit), wherever they were delivered from.
    struct Stats
    {
        uint64_t write_frame_ns = 0, wait_consumed_ns = 0, copy_ns = 0, slot_wait_ns = 0;
        uint64_t append_ns = 0, sink_ns = 0, units = 0;
    };
    const Stats& stats() const { return stats_; }

    // pinned host bytes held (batch buffers + unit buffers)
    size_t host_bytes() const
    {
        size_t n = in_.size() * 2 * size_t(opt_.batch_frames) * frame_bytes_;
        for (const Level& L : levels_)
            for (const auto& s : L.slots)
                n += s->cap + L.chunks_per_band;
        return n;
    }

    // One level-0 frame (frame_bytes bytes), to the stage that owns its z
    // plane.  Appends a full batch, or a slab run's last frames.
    aqz_status write_frame(const void* frame)
    {
        if (status_ != AQZ_STATUS_SUCCESS)
            return status_;
        Timed tw(stats_.write_frame_ns);
        uint32_t r = 0;
        bool run_end = false;
        if (st_.size() > 1) {
            const uint32_t z = uint32_t(accepted_ % plan_.planes);
            while (z >= plan_.end[r])
                ++r;
            run_end = z + 1 == plan_.end[r];
        }
        Input& in = in_[r];
        if (in.n == 0) {
            // refill only once the stage has read this buffer's last batch
            Timed t(stats_.wait_consumed_ns);
            const aqz_status s = aqz_stage_wait_consumed(st_[r], in.end[in.cur]);
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
        }
        Level* L0 = levels_.empty() || !levels_[0].host ? nullptr : &levels_[0];
        if (L0) {
            const aqz_status s = begin_host_unit_();
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
        }
        {
            Timed t(stats_.copy_ns);
            copy_frame_(in.buf[in.cur] + size_t(in.n) * frame_bytes_, frame, L0);
        }
        if (split_err_ != AQZ_STATUS_SUCCESS)
            return status_ = split_err_;
        ++in.n;
        ++in.appended;
        ++accepted_;
        if (L0 && accepted_ == host_.hi) {
            const aqz_status s = deliver_host_unit_(true);
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
        }
        if (in.n == opt_.batch_frames || run_end)
            return append_batch_(r);
        // units whose copies landed meanwhile go to the sink now
        return retire_(false);
    }

    // MultiscaleArray::close_ (multiscale.array.cpp:112-135): the partial
    // batches, the zero-filled remainder of every level's last layer (chunk.
    // cpp:8-15) and every remaining unit (Array::close_ flushes them,
    // array.cpp:374-424).
    aqz_status close()
    {
        if (status_ != AQZ_STATUS_SUCCESS)
            return status_;
        for (uint32_t r = 0; r < st_.size(); ++r) {
            const aqz_status s = append_batch_(r, false);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
        }
        for (aqz_stage* st : st_) {
            const aqz_status s = aqz_stage_finalize(st);
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
        }
        if (!levels_.empty() && levels_[0].host) {
            const aqz_status s = close_host_layer_();
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
        }
        aqz_status s = issue_(true);
        if (s == AQZ_STATUS_SUCCESS)
            s = drain_();
        if (s != AQZ_STATUS_SUCCESS)
            return status_ = s;
        for (Level& L : levels_)
            for (auto& sl : L.slots)
                wait_pins_(*sl);
        return AQZ_STATUS_SUCCESS;
    }

  private:
    struct Input // a stage's pinned double buffer of frames
    {
        uint8_t* buf[2] = { nullptr, nullptr };
        uint64_t end[2] = { 0, 0 }; // frames appended to the stage with each buffer
        int cur = 0;
        uint32_t n = 0;             // frames in buf[cur]
        uint64_t appended = 0;      // frames given to this stage (batched or not)
    };
    struct Slot
    {
        uint8_t* buf = nullptr;
        uint8_t* has = nullptr;
        size_t cap = 0;
        std::vector<aqz_chunk_entry> ent;
        std::atomic<int> pins{ 0 };
        bool busy = false; // compressing, or its copy in flight
        bool padding_clean = true; // host split: ragged padding is zero
    };
    struct Level
    {
        aqz_level_layout lay{};
        bool compressed = false;
        uint32_t n_bands = 1, chunks_per_band = 0;
        uint64_t frames_per_band = 0;
        uint32_t planes = 0; // z planes of the level (slab mode)
        bool host = false;   // level 0 split on the host (level0_on_host)
        bool ragged_last_band = false;
        uint64_t layer = 0;  // next unit to hand off: (layer, band)
        uint32_t band = 0;
        std::vector<std::unique_ptr<Slot>> slots;
        uint32_t next = 0;
    };
    struct Pending
    {
        uint32_t level, slot, owner;
        uint64_t layer;
        uint32_t band;
        uint64_t frames;
        bool complete;
        uint64_t ticket = 0; // 0: compression issued, frames not copied yet
    };

    static aqz_status worse(aqz_status a, aqz_status b)
    {
        return a != AQZ_STATUS_SUCCESS ? a : b;
    }

    // adds the scope's duration to a Stats counter
    struct Timed
    {
        uint64_t& acc;
        std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
        explicit Timed(uint64_t& a)
          : acc(a)
        {
        }
        ~Timed()
        {
            acc += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0)
                              .count());
        }
    };
    aqz_status to_sink_(Unit& u)
    {
        Timed t(stats_.sink_ns);
        ++stats_.units;
        return sink_.unit(u);
    }

    static void wait_pins_(Slot& s)
    {
        for (int v = s.pins.load(); v != 0; v = s.pins.load())
            s.pins.wait(v);
    }

    // ---- frame copy into the pinned batch, split over copy_threads ----------
    // With the host split of level 0 (split != null) each thread also splits
    // the rows it copied, from the caller's frame while they are in cache.
    void copy_frame_(uint8_t* dst, const void* src, Level* split)
    {
        const size_t nt = copiers_.size() + 1;
        csplit_ = split;
        if (nt == 1 || frame_bytes_ < (size_t(1) << 20)) {
            cdst_ = dst;
            csrc_ = static_cast<const uint8_t*>(src);
            copy_rows_(0, split ? rows_ : 0);
            if (!split)
                std::memcpy(dst, src, frame_bytes_);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(cmu_);
            cdst_ = dst;
            csrc_ = static_cast<const uint8_t*>(src);
            cleft_ = uint32_t(nt - 1);
            ++cgen_;
        }
        ccv_.notify_all();
        copy_part_(0);
        std::unique_lock<std::mutex> lk(cmu_);
        cdone_cv_.wait(lk, [&] { return cleft_ == 0; });
    }
    void copy_part_(uint32_t t)
    {
        const size_t nt = copiers_.size() + 1;
        if (csplit_) {
            const uint32_t per = uint32_t((rows_ + nt - 1) / nt);
            const uint32_t a = std::min<uint32_t>(rows_, per * t);
            copy_rows_(a, std::min<uint32_t>(rows_, a + per));
            return;
        }
        const size_t per = (frame_bytes_ / nt + 4095) & ~size_t(4095);
        const size_t a = std::min(frame_bytes_, per * t);
        const size_t b = std::min(frame_bytes_, a + per);
        if (b > a)
            std::memcpy(cdst_ + a, csrc_ + a, b - a);
    }
    // rows [a, b) of the frame: copied into the batch and split into the
    // current level-0 unit in one pass (the library's streaming copy)
    void copy_rows_(uint32_t a, uint32_t b)
    {
        if (b > a)
            split_host_rows_(csrc_, accepted_, a, b, cdst_);
    }
    void split_host_rows_(const uint8_t* frame, uint64_t fid, uint32_t r0, uint32_t r1,
                          uint8_t* frame_copy = nullptr)
    {
        Level& L = levels_[0];
        Slot& slot = *L.slots[host_.slot];
        const aqz_status s = aqz_stage_split_level0_rows(
          st_[0], frame, fid, r0, r1, frame_copy, host_.band * L.chunks_per_band, slot.buf,
          slot.cap, slot.has, L.chunks_per_band);
        if (s != AQZ_STATUS_SUCCESS) {
            std::lock_guard<std::mutex> lk(emu_);
            split_err_ = s;
        }
    }
    void copier_(uint32_t t)
    {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(cmu_);
        for (;;) {
            ccv_.wait(lk, [&] { return cstop_ || cgen_ != seen; });
            if (cstop_)
                return;
            seen = cgen_;
            lk.unlock();
            copy_part_(t);
            lk.lock();
            if (--cleft_ == 0)
                cdone_cv_.notify_one();
        }
    }

    // ---- level 0 split on the host ------------------------------------------------
    // The unit (layer, band) frame accepted_ belongs to gets a host slot when
    // its first frame arrives; it is handed to the sink as soon as its last
    // frame is split (no copy to wait for).
    struct HostUnit
    {
        bool open = false;
        uint32_t slot = 0, band = 0;
        uint64_t layer = 0, lo = 0, hi = 0;
    };

    aqz_status begin_host_unit_()
    {
        if (host_.open)
            return AQZ_STATUS_SUCCESS;
        Level& L = levels_[0];
        const uint64_t F = L.lay.frames_per_layer;
        const uint32_t si = L.next;
        const aqz_status s = take_slot_(*L.slots[si]);
        if (s != AQZ_STATUS_SUCCESS)
            return s;
        Slot& slot = *L.slots[si];
        host_.open = true;
        host_.slot = si;
        host_.layer = L.layer;
        host_.band = L.band;
        host_.lo = L.layer * F + uint64_t(L.band) * L.frames_per_band;
        host_.hi = L.layer * F + std::min<uint64_t>((uint64_t(L.band) + 1) * L.frames_per_band, F);
        const bool ragged = L.ragged_last_band && L.band + 1 == L.n_bands;
        if (ragged && !slot.padding_clean)
            std::memset(slot.buf, 0, slot.cap);
        slot.padding_clean = ragged || L.n_bands == 1;
        std::memset(slot.has, 0, L.chunks_per_band);
        L.next = (L.next + 1) % uint32_t(L.slots.size());
        return AQZ_STATUS_SUCCESS;
    }

    // the open unit to the sink: its frames [lo, min(accepted, hi)) are
    // split; complete = all of them
    aqz_status deliver_host_unit_(bool complete)
    {
        Level& L = levels_[0];
        Slot& slot = *L.slots[host_.slot];
        Unit u;
        u.level = 0;
        u.layer = host_.layer;
        u.band = host_.band;
        u.n_bands = L.n_bands;
        u.c0 = host_.band * L.chunks_per_band;
        u.n_chunks = L.chunks_per_band;
        u.first = host_.lo;
        u.frames = std::min(accepted_, host_.hi) - std::min(accepted_, host_.lo);
        u.complete = complete;
        u.last_in_layer = host_.band + 1 == L.n_bands;
        u.bytes_per_chunk = L.lay.bytes_per_chunk;
        u.chunks = slot.buf;
        u.has_data = slot.has;
        u.lease = Lease(&slot.pins);
        host_.open = false;
        if (++L.band == L.n_bands) {
            L.band = 0;
            ++L.layer;
        }
        return to_sink_(u);
    }

    // close: the rest of level 0's last, partial layer -- its frames not
    // written are zero (the reference's zeroed chunks, chunk.cpp:8-15) --
    // unit by unit, as the device side hands off its finalized layer
    aqz_status close_host_layer_()
    {
        Level& L = levels_[0];
        const uint64_t F = L.lay.frames_per_layer;
        if (accepted_ <= L.layer * F && !host_.open)
            return AQZ_STATUS_SUCCESS;
        const uint64_t layer = L.layer;
        std::vector<uint8_t> zero;
        while (L.layer == layer) {
            aqz_status s = begin_host_unit_();
            if (s != AQZ_STATUS_SUCCESS)
                return s;
            for (uint64_t f = std::max(accepted_, host_.lo); f < host_.hi; ++f) {
                if (zero.empty())
                    zero.assign(frame_bytes_, 0);
                split_host_rows_(zero.data(), f, 0, rows_);
                if (split_err_ != AQZ_STATUS_SUCCESS)
                    return split_err_;
            }
            s = deliver_host_unit_(false);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
        }
        return AQZ_STATUS_SUCCESS;
    }

    // ---- batches and units ------------------------------------------------------
    aqz_status append_batch_(uint32_t r, bool hand_off = true)
    {
        Input& in = in_[r];
        if (in.n == 0)
            return AQZ_STATUS_SUCCESS;
        aqz_status s;
        {
            Timed t(stats_.append_ns);
            s = aqz_stage_append(st_[r], in.buf[in.cur], in.n, AQZ_MEM_HOST_PINNED);
        }
        if (s != AQZ_STATUS_SUCCESS)
            return status_ = s;
        in.end[in.cur] = in.appended;
        in.cur ^= 1;
        in.n = 0;
        if (!hand_off)
            return AQZ_STATUS_SUCCESS;
        aqz_status h = issue_(false);
        if (h == AQZ_STATUS_SUCCESS)
            h = retire_(false);
        return h == AQZ_STATUS_SUCCESS ? h : (status_ = h);
    }

    // Frames of level l written so far by the whole stream.  One stage: its
    // own count (any cascade, odd z included).  z slabs (a regular z
    // schedule): every level-0 plane appended, stack by stack.
    uint64_t written_(uint32_t l) const
    {
        if (st_.size() == 1)
            return aqz_stage_frames_written(st_[0], l);
        uint64_t n0 = 0;
        for (const Input& in : in_)
            n0 += in.appended - in.n; // given to its stage (a batch not yet appended is not)
        const uint64_t Z = plan_.planes, Zk = levels_[l].planes;
        const uint64_t shift = ctz_(uint32_t(Z / Zk));
        return (n0 / Z) * Zk + ((n0 % Z) >> shift);
    }
    static uint32_t ctz_(uint32_t v)
    {
        uint32_t n = 0;
        while (v > 1) {
            v >>= 1;
            ++n;
        }
        return n;
    }

    // The stage that assembles and hands off a unit, after the others'
    // frames of it were imported (z slabs; round robin over layers so the
    // assembly traffic and the codec work spread over the GPUs).  Frames of
    // the unit not yet appended (close) are zeroed there.
    aqz_status assemble_(uint32_t l, uint64_t layer, uint64_t lo, uint64_t hi,
                         uint64_t written, uint32_t& owner)
    {
        owner = 0;
        if (st_.size() == 1)
            return AQZ_STATUS_SUCCESS;
        const Level& L = levels_[l];
        const uint64_t F = L.lay.frames_per_layer;
        const uint32_t shift = ctz_(plan_.planes / L.planes);
        owner = uint32_t(layer % st_.size());
        for (uint64_t f = lo; f < hi;) {
            const uint32_t z = uint32_t(f % L.planes);
            uint32_t r = 0;
            while (z >= (plan_.end[r] >> shift))
                ++r;
            const uint64_t run_end = std::min<uint64_t>(hi, f - z + (plan_.end[r] >> shift));
            const uint64_t have = std::min(std::max(written, f), run_end); // [f, have) written
            if (r != owner && have > f) {
                const aqz_status s =
                  aqz_stage_import_frames(st_[owner], st_[r], l, layer, uint32_t(f - layer * F),
                                          uint32_t(have - f));
                if (s != AQZ_STATUS_SUCCESS)
                    return s;
            }
            if (run_end > have) {
                const aqz_status s =
                  aqz_stage_import_frames(st_[owner], nullptr, l, layer,
                                          uint32_t(have - layer * F), uint32_t(run_end - have));
                if (s != AQZ_STATUS_SUCCESS)
                    return s;
            }
            f = run_end;
        }
        return AQZ_STATUS_SUCCESS;
    }

    // Hand off every unit of every level whose frames are all written (final:
    // also every unit of each level's last, partially written layer).  Unit
    // (layer, band) covers the level's frames [layer F + band fpb,
    // layer F + min((band + 1) fpb, F)): the trailing band of a ragged dim 1
    // is complete with its layer (array.cpp:884-886).
    aqz_status issue_(bool final)
    {
        for (uint32_t l = 0; l < levels_.size(); ++l) {
            Level& L = levels_[l];
            if (L.host)
                continue; // split on the host, handed off as its frames arrive
            const uint64_t F = L.lay.frames_per_layer;
            for (;;) {
                const uint64_t written = written_(l);
                const uint64_t lo = L.layer * F + uint64_t(L.band) * L.frames_per_band;
                const uint64_t hi =
                  L.layer * F + std::min<uint64_t>((uint64_t(L.band) + 1) * L.frames_per_band, F);
                const bool complete = written >= hi;
                if (!complete && !(final && written > L.layer * F))
                    break;
                const uint32_t si = L.next;
                aqz_status s = take_slot_(*L.slots[si]);
                if (s != AQZ_STATUS_SUCCESS)
                    return s;
                Slot& slot = *L.slots[si];
                uint32_t owner = 0;
                // a compressed unit is the whole layer
                s = L.compressed ? assemble_(l, L.layer, L.layer * F, (L.layer + 1) * F, written,
                                             owner)
                                 : assemble_(l, L.layer, lo, hi, written, owner);
                if (s != AQZ_STATUS_SUCCESS)
                    return s;
                aqz_stage* st = st_[owner];
                Pending p{ l, si, owner, L.layer, L.band,
                           std::min(written, hi) - std::min(written, lo), complete, 0 };
                if (L.compressed) {
                    // the previous occupant of this layer's device frame slot
                    // must be on its way out before the slot is rewritten
                    s = flush_compressions_(l, L.layer, owner);
                    if (s == AQZ_STATUS_SUCCESS)
                        s = aqz_stage_compress_layer(st, l, L.layer, &opt_.comp);
                    if (s != AQZ_STATUS_SUCCESS)
                        return s;
                    compressing_.push_back(p);
                } else {
                    const size_t cap = size_t(L.lay.bytes_per_chunk) * L.chunks_per_band;
                    s = L.n_bands > 1
                          ? aqz_stage_copy_band_async(st, l, L.layer, L.band, slot.buf, cap,
                                                      slot.has, L.chunks_per_band)
                          : aqz_stage_copy_layer_async(st, l, L.layer, slot.buf, cap, slot.has,
                                                       L.chunks_per_band);
                    if (s != AQZ_STATUS_SUCCESS)
                        return s;
                    p.ticket = aqz_stage_last_ticket(st);
                    inflight_.push_back(p);
                }
                slot.busy = true;
                L.next = (L.next + 1) % uint32_t(L.slots.size());
                if (++L.band == L.n_bands) {
                    L.band = 0;
                    ++L.layer;
                }
            }
        }
        return advance_compressions_(false);
    }

    // Wait until a host slot is free: neither compressing nor in flight, and
    // no lease on it.
    aqz_status take_slot_(Slot& slot)
    {
        Timed t(stats_.slot_wait_ns);
        while (slot.busy) {
            const aqz_status s = progress_(true);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
        }
        wait_pins_(slot);
        return AQZ_STATUS_SUCCESS;
    }

    // Compressed layers of level l on stage `owner` that share the device
    // frame slot of `layer` (layer - layer_slots and earlier) get their D2H
    // issued.
    aqz_status flush_compressions_(uint32_t l, uint64_t layer, uint32_t owner)
    {
        const uint64_t ns = std::max<uint32_t>(1, levels_[l].lay.layer_slots);
        for (;;) {
            bool found = false;
            for (const Pending& p : compressing_)
                found |= p.level == l && p.owner == owner && p.layer + ns <= layer;
            if (!found)
                return AQZ_STATUS_SUCCESS;
            const aqz_status s = advance_compressions_(true);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
        }
    }

    // Finished compressions (oldest first; block: the oldest one at least)
    // get their frames copied D2H.
    aqz_status advance_compressions_(bool block)
    {
        while (!compressing_.empty()) {
            Pending p = compressing_.front();
            aqz_stage* st = st_[p.owner];
            if (!block) {
                int32_t done = 0;
                const aqz_status s = aqz_stage_compression_done(st, p.level, p.layer, &done);
                if (s != AQZ_STATUS_SUCCESS)
                    return s;
                if (!done)
                    return AQZ_STATUS_SUCCESS;
            }
            Slot& slot = *levels_[p.level].slots[p.slot];
            // the entries now: the device frame slot may take a newer layer
            // once this copy is issued (the stage orders the device side)
            aqz_status s = aqz_stage_compressed_entries(st, p.level, p.layer, slot.ent.data(),
                                                        slot.ent.size());
            if (s == AQZ_STATUS_SUCCESS)
                s = aqz_stage_copy_compressed_async(st, p.level, p.layer, slot.buf, slot.cap);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
            p.ticket = aqz_stage_last_ticket(st);
            compressing_.pop_front();
            inflight_.push_back(p);
            block = false;
        }
        return AQZ_STATUS_SUCCESS;
    }

    // One step: landed units to the sink; with block, wait for the oldest
    // copy (or compression) when nothing has landed.
    aqz_status progress_(bool block)
    {
        aqz_status s = advance_compressions_(false);
        if (s != AQZ_STATUS_SUCCESS)
            return s;
        const size_t before = inflight_.size() + compressing_.size();
        s = retire_(false);
        if (s != AQZ_STATUS_SUCCESS || !block)
            return s;
        if (inflight_.size() + compressing_.size() < before)
            return AQZ_STATUS_SUCCESS;
        if (!inflight_.empty())
            return retire_one_(true);
        if (!compressing_.empty())
            return advance_compressions_(true);
        return AQZ_STATUS_INTERNAL_ERROR; // waiting for a slot nothing holds
    }

    // Deliver the oldest in-flight unit (wait: block until its copy landed;
    // else only if it has).  A stage's tickets complete in issue order, and
    // per level units are issued in frame order.
    aqz_status retire_one_(bool wait)
    {
        if (inflight_.empty())
            return AQZ_STATUS_SUCCESS;
        const Pending p = inflight_.front();
        aqz_stage* st = st_[p.owner];
        if (wait) {
            const aqz_status s = aqz_stage_wait_ticket(st, p.ticket);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
        } else if (aqz_stage_copies_completed(st) < p.ticket) {
            return AQZ_STATUS_SUCCESS;
        }
        inflight_.pop_front();
        Level& L = levels_[p.level];
        Slot& slot = *L.slots[p.slot];
        Unit u;
        u.level = p.level;
        u.layer = p.layer;
        u.band = p.band;
        u.n_bands = L.n_bands;
        u.c0 = p.band * L.chunks_per_band;
        u.n_chunks = L.chunks_per_band;
        u.first = p.layer * L.lay.frames_per_layer + uint64_t(p.band) * L.frames_per_band;
        u.frames = p.frames;
        u.complete = p.complete;
        u.last_in_layer = p.band + 1 == L.n_bands;
        u.bytes_per_chunk = L.lay.bytes_per_chunk;
        if (L.compressed) {
            u.data = slot.buf;
            u.entries = slot.ent.data();
        } else {
            u.chunks = slot.buf;
            u.has_data = slot.has;
        }
        u.lease = Lease(&slot.pins);
        slot.busy = false;
        return to_sink_(u);
    }

    aqz_status retire_(bool wait_all)
    {
        while (!inflight_.empty()) {
            const size_t before = inflight_.size();
            const aqz_status s = retire_one_(wait_all);
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
            if (inflight_.size() == before) // the oldest copy is still in flight
                break;
        }
        return AQZ_STATUS_SUCCESS;
    }

    aqz_status drain_()
    {
        while (!compressing_.empty() || !inflight_.empty()) {
            aqz_status s = advance_compressions_(inflight_.empty());
            if (s == AQZ_STATUS_SUCCESS)
                s = retire_(true);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
        }
        return AQZ_STATUS_SUCCESS;
    }

    std::vector<aqz_stage*> st_;
    SlabPlan plan_;
    const uint64_t frame_bytes_;
    HandoffOptions opt_;
    HandoffSink& sink_;
    aqz_status status_ = AQZ_STATUS_SUCCESS;
    std::vector<Input> in_;
    uint64_t accepted_ = 0;
    std::vector<Level> levels_;
    std::deque<Pending> compressing_; // compression issued, in issue order
    std::deque<Pending> inflight_;    // copies issued, in issue order
    Stats stats_;
    // level 0 split on the host
    HostUnit host_;
    uint32_t rows_ = 0;     // level-0 rows per frame
    uint64_t row_bytes_ = 0;
    Level* csplit_ = nullptr;
    std::mutex emu_;
    aqz_status split_err_ = AQZ_STATUS_SUCCESS;
    // frame copy threads
    std::vector<std::thread> copiers_;
    std::mutex cmu_;
    std::condition_variable ccv_, cdone_cv_;
    bool cstop_ = false;
    uint64_t cgen_ = 0;
    uint32_t cleft_ = 0;
    uint8_t* cdst_ = nullptr;
    const uint8_t* csrc_ = nullptr;
};

} // namespace aqz_binding
