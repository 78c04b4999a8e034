// multiscale.array.gpu.cpp -- the reference-side binding of the MI355X stage.
//
// This is the file a maintainer adds to acquire-zarr's src/streaming/ (built
// when ZARR_WITH_AQZ is on).  It is complete: the
// CPU suite compiles it with -fsyntax-only against the reference's own
// headers (tests/test_abi_pin_cpu.py), so every member it touches exists
// with the type used here.
//
//   GpuArray            : zarr::Array (array.hh:12-104) whose chunks arrive
//                         from the GPU -- raw, or already compressed on the
//                         device -- instead of from write_frame_to_chunks_
//                         (array.cpp:507-622) and Chunk::compress_and_take_
//                         buffer (chunk.cpp:78-106).  Each chunk goes to its
//                         Shard with write_chunk / skip_chunk on the thread
//                         pool, with the reference's retries, ragged-padding
//                         skips, layer advance and rollover (array.cpp:
//                         664-908).
//   GpuMultiscaleArray  : zarr::MultiscaleArray (multiscale.array.hh:9-65)
//                         whose write_frame (multiscale.array.cpp:57-74)
//                         appends frames to the aqz stage -- level-0 tile
//                         split, Downsampler::add_frame, every level's tile
//                         split and the chunk codec on the device -- and
//                         hands every unit to the per-level GpuArrays through
//                         aqz_handoff.hh.  Metadata (zarr.json, OME
//                         multiscales) stays the reference's: the base class
//                         keeps its Downsampler for level geometry and
//                         get_metadata(), which aqz reproduces byte for byte.
//   make_gpu_multiscale_array : the hook ZarrStream_s::configure_array_
//                         (zarr.stream.cpp:1231-1279) calls before
//                         zarr::make_array; nullptr = the reference path.
#include "array.hh"
#include "macros.hh"
#include "multiscale.array.hh"
#include "zarr.common.hh"

#include "aqz_gpu.h"
#include "aqz_handoff.hh"

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace zarr {

// The reference classes the binding derives from.  tests/native/
// binding_exec.cpp defines AQZ_BINDING_TEST_BASES and test doubles under
// these two names (their members restated from array.cpp / shard.cpp /
// multiscale.array.cpp, whose definitions do not build in that harness), so
// that this file's code -- every line of it, unchanged -- runs on the GPU
// against them.
#ifndef AQZ_BINDING_TEST_BASES
using GpuArrayBase = Array;
using GpuMultiscaleArrayBase = MultiscaleArray;
#endif

// ZarrCompressionSettings as the reference applies them (compression_params,
// zarr.stream.cpp:191-208; chunk.cpp:78-106) -> the device codec.
inline aqz_compression
aqz_codec_for(const std::optional<CompressionParams>& params)
{
    aqz_compression c{ AQZ_CODEC_NONE, 0, 0 };
    if (!params)
        return c;
    if (const auto* b = std::get_if<BloscCompressionParams>(&*params)) {
        c.codec = b->codec_id == "zstd" ? AQZ_CODEC_BLOSC_ZSTD : AQZ_CODEC_BLOSC_LZ4;
        c.clevel = b->clevel;
        c.shuffle = b->shuffle;
    } else if (const auto* z = std::get_if<ZstdCompressionParams>(&*params)) {
        c.codec = AQZ_CODEC_ZSTD;
        c.clevel = z->level;
    }
    return c;
}

// ZarrCompressionSettings -> the array's CompressionParams, as the stream
// builds them (make_compression_params, zarr.stream.cpp:191-208): the
// compressor field decides, the codec only names blosc's inner codec.
inline std::optional<CompressionParams>
compression_params_of(const ZarrCompressionSettings* s)
{
    if (!s || s->compressor == ZarrCompressor_None)
        return std::nullopt;
    if (s->compressor == ZarrCompressor_Blosc1)
        return BloscCompressionParams(blosc_codec_to_string(s->codec), s->level, s->shuffle);
    if (s->compressor == ZarrCompressor_Zstd)
        return ZstdCompressionParams{ s->level };
    return std::nullopt;
}

// The reference's ArrayDimensions as the router's ShardMap.
class RefShardMap final : public aqz_binding::ShardMap
{
  public:
    explicit RefShardMap(std::shared_ptr<ArrayDimensions> dims)
      : dims_(std::move(dims))
    {
    }
    uint32_t chunks_in_memory() const override { return dims_->number_of_chunks_in_memory(); }
    uint32_t number_of_shards() const override { return dims_->number_of_shards(); }
    uint32_t shard_index_for_chunk(uint32_t c) const override
    {
        return dims_->shard_index_for_chunk(c);
    }
    uint32_t shard_internal_index(uint32_t c) const override
    {
        return dims_->shard_internal_index(c);
    }
    std::vector<uint32_t> skipped_internal_indices(uint32_t shard,
                                                   uint32_t layer) const override
    {
        return dims_->skipped_internal_indices_for_shard_layer(shard, layer);
    }

  private:
    std::shared_ptr<ArrayDimensions> dims_;
};

class GpuArray final
  : public GpuArrayBase
  , private aqz_binding::ShardWriter
{
  public:
    GpuArray(std::shared_ptr<ArrayConfig> config,
             std::shared_ptr<ThreadPool> thread_pool,
             std::shared_ptr<FileHandlePool> file_handle_pool,
             std::shared_ptr<S3ConnectionPool> s3_connection_pool)
      : GpuArrayBase(config, thread_pool, file_handle_pool, s3_connection_pool)
      , map_(config_->dimensions)
      , router_(map_)
    {
    }

    // Every chunk of a handed-off unit to its shard through the shared
    // router (aqz_handoff.hh ShardRouter::route: the chunk jobs of
    // Array::dispatch_chunk_job_, array.cpp:664-760, with the bytes already
    // made -- raw when no codec is configured, else the device's frame --
    // Shard::skip_chunk for a chunk without data, and the ragged-padding
    // skips on a layer's last unit, array.cpp:771-790, 852-862).
    aqz_status write_unit(const aqz_binding::Unit& u)
    {
        if (data_paths_.empty())
            make_shards_();
        return router_.route(u, *this);
    }

    // `frames` more frames are in the shards: the tail of Array::write_frame
    // (array.cpp:196-219), then the router's layer advance or rollover
    // (ShardRouter::commit: compress_and_flush_data_ :799-803,
    // flush_completed_bands_ :880-898).  The last, partial layer at close
    // is already written, so close_ has nothing to flush.
    // The counters are aqz_binding::ArrayLedger's (the code the GPU replay
    // runs and checks against the reference's per-frame rules), mirrored
    // into the reference's members before should_rollover_ reads them.
    WriteResult commit_unit(const aqz_binding::Unit& u)
    {
        if (!ledger_.commit(u, bytes_per_frame_, max_bytes_))
            return WriteResult::OutOfBounds;
        total_bytes_written_ = ledger_.total_bytes_written;
        last_successful_frame_id_ = ledger_.last_successful_frame_id;
        bytes_to_flush_ = ledger_.bytes_to_flush;
        flushed_band_count_ = ledger_.flushed_band_count;
        router_.commit(u, *this);
        current_layer_ = router_.current_layer();
        return WriteResult::Ok;
    }

  private:
    // aqz_binding::ShardWriter: the reference's own jobs and rollover
    void write_chunk(uint32_t shard, uint32_t internal, uint32_t chunk, const uint8_t* bytes,
                     size_t n, const aqz_binding::Lease& lease) override
    {
        dispatch_bytes_job_(shards_[shard], chunk, internal, shard, bytes, n, lease);
    }
    void skip_chunk(uint32_t shard, uint32_t internal, uint32_t) override
    {
        dispatch_skip_(shards_[shard], internal, shard);
    }
    bool should_rollover() override { return should_rollover_(); }
    void rollover() override
    {
        rollover_();
        CHECK(write_metadata_());
    }

    RefShardMap map_;
    aqz_binding::ShardRouter router_;
    aqz_binding::ArrayLedger ledger_;

    // std::shared_ptr<Shard> (array.hh:43)
    using ShardPtr = decltype(shards_)::value_type;

    // A writer job ends: write_counter_ drops under write_counter_mutex_, the
    // mutex Array::close_ checks its predicate under (array.cpp:390-392), so
    // close_ cannot miss the last notification.  The reference's own jobs
    // decrement without it (array.cpp:649-650, 743-744): a job that ends
    // between close_'s predicate check and its wait is a lost wake-up, and
    // close_ then waits forever -- seen here as an occasional stalled close
    // of the binding harness, which is why the binding runs its skips with
    // its own jobs too instead of Array::dispatch_skip_job_.
    void job_done_()
    {
        {
            std::lock_guard<std::mutex> lk(write_counter_mutex_);
            write_counter_.fetch_sub(1);
        }
        write_counter_cv_.notify_all();
    }

    // Array::dispatch_skip_job_ (array.cpp:625-662) with job_done_
    void dispatch_skip_(ShardPtr shard, uint32_t internal_idx, uint32_t shard_idx)
    {
        write_counter_.fetch_add(1);
        auto job = [this, shard, internal_idx, shard_idx](std::string& err) {
            ThreadPool::TaskResult result = ThreadPool::TaskResult::Success;
            try {
                if (!shard->skip_chunk(internal_idx)) {
                    err = "Failed to skip chunk " + std::to_string(internal_idx) + " of shard " +
                          std::to_string(shard_idx);
                    result = ThreadPool::TaskResult::Fatal;
                }
            } catch (const std::exception& exc) {
                err = std::string("Failed skipping chunk: ") + exc.what();
                result = ThreadPool::TaskResult::Fatal;
            }
            job_done_();
            return result;
        };
        if (thread_pool_->n_threads() == 1 || !thread_pool_->push_job(job)) {
            if (!thread_pool_->execute_job(std::move(job)))
                LOG_ERROR("Failed to skip chunk ", internal_idx, " of shard ", shard_idx);
        }
    }

    void dispatch_bytes_job_(ShardPtr shard,
                             uint32_t chunk_idx,
                             uint32_t internal_idx,
                             uint32_t shard_idx,
                             const uint8_t* bytes,
                             size_t nbytes,
                             aqz_binding::Lease lease)
    {
        write_counter_.fetch_add(1);
        auto job = [this, shard, chunk_idx, internal_idx, shard_idx, bytes, nbytes,
                    lease = std::move(lease)](std::string& err) mutable {
            ThreadPool::TaskResult result = ThreadPool::TaskResult::Success;
            try {
                // Shard::write_chunk takes a vector (shard.hh:38); the copy
                // out of the pinned hand-off buffer runs here, on the pool
                const std::vector<uint8_t> buffer(bytes, bytes + nbytes);
                lease.release();
                constexpr size_t n_retries = 3;
                bool ok = false;
                for (size_t retry = 0; retry < n_retries && !ok; ++retry) {
                    ok = shard->write_chunk(internal_idx, buffer);
                    if (!ok)
                        std::this_thread::sleep_for(std::chrono::milliseconds(
                          static_cast<int>(std::pow(10, retry))));
                }
                if (!ok) {
                    err = "Failed to write chunk " + std::to_string(chunk_idx) + " of shard " +
                          std::to_string(shard_idx) + " after " + std::to_string(n_retries) +
                          " attempts";
                    result = ThreadPool::TaskResult::Fatal;
                }
            } catch (const std::exception& exc) {
                err = std::string("Failed to write chunk: ") + exc.what();
                result = ThreadPool::TaskResult::Fatal;
            }
            job_done_();
            return result;
        };
        if (thread_pool_->n_threads() == 1 || !thread_pool_->push_job(job)) {
            if (!thread_pool_->execute_job_with_retry(std::move(job), 2))
                LOG_ERROR("Failed to write chunk ", chunk_idx, " (internal index ",
                          internal_idx, ") of shard ", shard_idx);
        }
    }
};

class GpuMultiscaleArray final
  : public GpuMultiscaleArrayBase
  , private aqz_binding::HandoffSink
{
  public:
    // settings: the ZarrArraySettings the stream was configured with
    // (acquisition-order dims + storage order, zarr.types.h:157-169);
    // devices: HIP device ordinals (aqz_binding::select_device), one per
    // z slab of `plan` (one device: no slabs).
    GpuMultiscaleArray(std::shared_ptr<ArrayConfig> config,
                       std::shared_ptr<ThreadPool> thread_pool,
                       std::shared_ptr<FileHandlePool> file_handle_pool,
                       std::shared_ptr<S3ConnectionPool> s3_connection_pool,
                       const ZarrArraySettings& settings,
                       std::vector<int32_t> devices,
                       const aqz_binding::SlabPlan& plan = {},
                       uint32_t batch_frames = 64,
                       uint32_t host_slots = 3)
      : GpuMultiscaleArrayBase(config, thread_pool, file_handle_pool, s3_connection_pool)
    {
        EXPECT(downsampler_ != nullptr, "GpuMultiscaleArray needs a downsampling method");
        // per-level writers that take GPU-made chunks (create_arrays_,
        // multiscale.array.cpp:137-159, with GpuArray for Array)
        gpu_arrays_.clear();
        for (const auto& [lod, cfg] : downsampler_->writer_configurations()) {
            auto a = std::make_unique<GpuArray>(cfg, thread_pool_, file_handle_pool_,
                                                s3_connection_pool_);
            if (gpu_arrays_.size() <= size_t(lod))
                gpu_arrays_.resize(lod + 1, nullptr);
            gpu_arrays_[lod] = a.get();
            arrays_[lod] = std::move(a);
        }
        // every level's CPU Array was replaced (create_arrays_ made one per
        // writer configuration, multiscale.array.cpp:137-159)
        EXPECT(gpu_arrays_.size() == arrays_.size(), "a level without a GpuArray");
        for (size_t l = 0; l < arrays_.size(); ++l)
            EXPECT(gpu_arrays_[l] != nullptr && arrays_[l].get() == gpu_arrays_[l],
                   "level ", l, " still has a CPU Array");

        dims_.resize(settings.dimension_count);
        for (size_t i = 0; i < settings.dimension_count; ++i) {
            const ZarrDimensionProperties& p = settings.dimensions[i];
            dims_[i] = aqz_dimension{ int32_t(p.type), p.array_size_px, p.chunk_size_px,
                                      p.shard_size_chunks };
        }
        aqz_array_desc desc{ dims_.data(),
                             dims_.size(),
                             int32_t(settings.data_type),
                             1,
                             int32_t(*config_->downsampling_method),
                             settings.max_levels,
                             settings.storage_dimension_order,
                             0 };
        EXPECT(!devices.empty() && (devices.size() == 1 || plan.begin.size() == devices.size()),
               "one device per z slab");
        const aqz_compression comp = aqz_codec_for(config_->compression_params);
        // a raw hand-off splits level 0 on the host, in the copy threads'
        // pass over each frame: only levels >= 1 come back over PCIe
        // 
        const bool level0_host = aqz_binding::level0_on_host_for(desc, comp);
        for (size_t r = 0; r < devices.size(); ++r) {
            desc.device = devices[r];
            aqz_stage_options opt{};
            opt.max_batch_frames = batch_frames;
            opt.layer_slots = 2;
            opt.level0_split_on_host = level0_host ? 1u : 0u;
            // the library maps the chunk-layer rings from 2 MiB virtual-
            // memory pieces, where the fused kernels run in the fast band on
            // most boxes; the arena is timed once against a streaming probe
            // of the same memory, and only where it runs more than 3% under
            // that is one fresh arena tried (the
            // transient peak, one more ring set and a batch of random frames,
            // is in aqz_stage_estimate_memory)
            opt.placement_tries = 2;
            if (devices.size() > 1) {
                opt.z_slab_begin = plan.begin[r];
                opt.z_slab_end = plan.end[r];
            }
            aqz_stage* st = nullptr;
            EXPECT(aqz_stage_create(&desc, &opt, &st) == AQZ_STATUS_SUCCESS,
                   "aqz_stage_create failed: ", aqz_last_error());
            stages_.push_back(st);
            EXPECT(aqz_stage_n_levels(st) == arrays_.size(),
                   "level count differs from the Downsampler's");
        }
        aqz_binding::HandoffOptions ho;
        ho.batch_frames = batch_frames;
        ho.host_slots = host_slots;
        ho.comp = comp;
        ho.level0_on_host = level0_host;
        aqz_binding::HandoffSink& sink = *this;
        handoff_ = std::make_unique<aqz_binding::Handoff>(
          stages_, devices.size() > 1 ? plan : aqz_binding::SlabPlan{}, bytes_per_frame_, ho,
          sink);
        EXPECT(handoff_->status() == AQZ_STATUS_SUCCESS, "aqz hand-off buffers: ",
               aqz_status_message(handoff_->status()));
    }

    ~GpuMultiscaleArray() override
    {
        handoff_.reset();
        for (aqz_stage* st : stages_)
            aqz_stage_destroy(st);
    }

    // Host memory, as ZarrStream_get_current_memory_usage sums it
    // (zarr.stream.cpp:1057-1068): the base array's plus the stages' pinned
    // memory and the hand-off's pinned buffers.  Device memory is not host
    // memory: it is reported by device_memory_usage() instead.
    size_t memory_usage() const noexcept override
    {
        size_t pinned = 0;
        for (aqz_stage* st : stages_) {
            aqz_memory_usage m{};
            (void)aqz_stage_memory_usage(st, &m);
            pinned += m.pinned_bytes;
        }
        return GpuMultiscaleArrayBase::memory_usage() + pinned + handoff_->host_bytes();
    }

    // Sidecar (not part of the reference's interface): HBM the stages hold
    // (aqz_stage_memory_usage), for a caller that reports device memory
    // next to the host figure.
    size_t device_memory_usage() const noexcept
    {
        size_t dev = 0;
        for (aqz_stage* st : stages_) {
            aqz_memory_usage m{};
            (void)aqz_stage_memory_usage(st, &m);
            dev += m.device_bytes;
        }
        return dev;
    }

    // MultiscaleArray::write_frame (multiscale.array.cpp:57-74) with the
    // checks of Array::write_frame (array.cpp:160-189).  The hand-off
    // batches frames into pinned memory; nothing here waits for the GPU
    // except to refill a batch buffer the stage has not read yet.
    [[nodiscard]] WriteResult write_frame(std::vector<uint8_t>& frame,
                                          size_t& bytes_written,
                                          uint64_t frame_id) override
    {
        bytes_written = 0;
        if (frame.size() != bytes_per_frame_)
            return WriteResult::FrameSizeMismatch;
        if (frame_id != handoff_->frames_accepted())
            return WriteResult::FrameOutOfOrder;
        const uint64_t max = arrays_[0]->max_bytes();
        if (max > 0 && (handoff_->frames_accepted() + 1) * bytes_per_frame_ > max)
            return WriteResult::OutOfBounds;
        const aqz_status s = handoff_->write_frame(frame.data());
        if (s == AQZ_STATUS_WRITE_OUT_OF_BOUNDS)
            return WriteResult::OutOfBounds;
        EXPECT(s == AQZ_STATUS_SUCCESS, "aqz stage: ", aqz_status_message(s), ": ",
               aqz_last_error());
        bytes_written = frame.size();
        return WriteResult::Ok;
    }

  protected:
    bool close_() override
    {
        try {
            const aqz_status s = handoff_->close();
            EXPECT(s == AQZ_STATUS_SUCCESS, "aqz stage: ", aqz_status_message(s), ": ",
                   aqz_last_error());
        } catch (const std::exception& exc) {
            LOG_ERROR("Failed to finalize the GPU stage: ", exc.what());
            return false;
        }
        return GpuMultiscaleArrayBase::close_();
    }

  private:
    // aqz_binding::HandoffSink: units land in frame order per level
    aqz_status unit(aqz_binding::Unit& u) override
    {
        try {
            const aqz_status s = gpu_arrays_[u.level]->write_unit(u);
            if (s != AQZ_STATUS_SUCCESS) {
                LOG_ERROR("A GPU chunk unit disagrees with the level's shard map");
                return s;
            }
            return gpu_arrays_[u.level]->commit_unit(u) == WriteResult::Ok
                     ? AQZ_STATUS_SUCCESS
                     : AQZ_STATUS_WRITE_OUT_OF_BOUNDS;
        } catch (const std::exception& exc) {
            LOG_ERROR("Failed to write a GPU chunk unit: ", exc.what());
            return AQZ_STATUS_INTERNAL_ERROR;
        }
    }

    std::vector<aqz_stage*> stages_;
    std::vector<aqz_dimension> dims_;
    std::vector<GpuArray*> gpu_arrays_;
    std::unique_ptr<aqz_binding::Handoff> handoff_;
};

// AQZ_Z_SLABS=N on a volume stream (a z Space dimension before y,
// acquisition storage order): the z-slab plan over N stages; an empty plan
// otherwise (one stage).
inline aqz_binding::SlabPlan
gpu_slab_plan(const ZarrArraySettings& settings)
{
    aqz_binding::SlabPlan plan;
    const uint32_t slabs = aqz_binding::slabs_from_env();
    const size_t nd = settings.dimension_count;
    bool identity = true;
    for (size_t i = 0; settings.storage_dimension_order && i < nd; ++i)
        identity &= settings.storage_dimension_order[i] == i;
    if (slabs > 1 && nd >= 4 && identity &&
        settings.dimensions[nd - 3].type == ZarrDimensionType_Space) {
        // level z extents: slab bounds must be multiples of 2^(z halvings)
        std::vector<aqz_dimension> d(nd);
        for (size_t i = 0; i < nd; ++i)
            d[i] = aqz_dimension{ int32_t(settings.dimensions[i].type),
                                  settings.dimensions[i].array_size_px,
                                  settings.dimensions[i].chunk_size_px,
                                  settings.dimensions[i].shard_size_chunks };
        uint32_t nl = 0;
        if (aqz_pyramid_levels(d.data(), nd, settings.max_levels, &nl, nullptr, 0) ==
            AQZ_STATUS_SUCCESS) {
            std::vector<aqz_dimension> lv(size_t(nl) * nd);
            if (aqz_pyramid_levels(d.data(), nd, settings.max_levels, &nl, lv.data(),
                                   lv.size()) == AQZ_STATUS_SUCCESS) {
                const uint32_t z0 = lv[nd - 3].array_size_px;
                const uint32_t zl = lv[(nl - 1) * nd + nd - 3].array_size_px;
                plan = aqz_binding::plan_z_slabs(z0, slabs, zl ? z0 / zl : 0);
            }
        }
    }
    return plan;
}

// The binding's share of ZarrStreamSettings_estimate_max_memory_usage
// (acquire.zarr.cpp:216-314) for one array the GPU path would take (the
// same conditions as make_gpu_multiscale_array): host_bytes is added to
// *usage there -- the pinned hand-off and stage buffers, on top of the
// reference's own terms for the array, which stay -- and device_bytes is
// the HBM it needs, for a caller that reports it beside (INTEGRATION.md
// section 2).  {0, 0} for an array that stays on the CPU path.
inline aqz_binding::MemoryEstimate
estimate_gpu_array_memory(const ZarrArraySettings& settings,
                          uint32_t batch_frames = 64,
                          uint32_t host_slots = 3)
{
    aqz_binding::MemoryEstimate m{};
    int32_t n = 0;
    const char* e = std::getenv("AQZ_DEVICE");
    // make_gpu_multiscale_array's conditions (a multiscale array with a
    // downsampling method, a visible device, AQZ_DEVICE not off)
    if (!settings.multiscale || settings.downsampling_method >= ZarrDownsamplingMethodCount ||
        aqz_device_count(&n) != AQZ_STATUS_SUCCESS || n <= 0 ||
        (e && (std::string(e) == "off" || std::string(e) == "-1")))
        return m;
    std::vector<aqz_dimension> dims(settings.dimension_count);
    for (size_t i = 0; i < dims.size(); ++i) {
        const ZarrDimensionProperties& p = settings.dimensions[i];
        dims[i] = aqz_dimension{ int32_t(p.type), p.array_size_px, p.chunk_size_px,
                                 p.shard_size_chunks };
    }
    const aqz_array_desc desc{ dims.data(),
                               dims.size(),
                               int32_t(settings.data_type),
                               1,
                               int32_t(settings.downsampling_method),
                               settings.max_levels,
                               settings.storage_dimension_order,
                               0 };
    // the codec the array gets (its CompressionParams, as the stream builds
    // them) and, from it, the level-0 side -- as GpuMultiscaleArray decides
    const aqz_compression comp = aqz_codec_for(compression_params_of(settings.compression_settings));
    const bool level0_host = aqz_binding::level0_on_host_for(desc, comp);
    aqz_stage_options opt{};
    opt.max_batch_frames = batch_frames;
    opt.layer_slots = 2;
    opt.placement_tries = 2; // as GpuMultiscaleArray creates its stages
    opt.level0_split_on_host = level0_host ? 1u : 0u;
    aqz_binding::HandoffOptions ho;
    ho.batch_frames = batch_frames;
    ho.host_slots = host_slots;
    ho.comp = comp;
    ho.level0_on_host = level0_host;
    const auto plan = gpu_slab_plan(settings);
    const uint32_t stages = uint32_t(std::max<size_t>(1, plan.begin.size()));
    if (aqz_binding::estimate_memory(desc, opt, ho, stages, &m) != AQZ_STATUS_SUCCESS)
        return aqz_binding::MemoryEstimate{};
    return m;
}

// The hook of ZarrStream_s::configure_array_ (zarr.stream.cpp:1231-1279):
//
//     #ifdef ZARR_WITH_AQZ
//         output->array = zarr::make_gpu_multiscale_array(
//           config, thread_pool_, file_handle_pool_, s3_connection_pool_, *settings);
//         if (!output->array)
//     #endif
//         output->array = zarr::make_array(config, thread_pool_, ...);
//
// A multiscale array gets the GPU stage on the device AQZ_DEVICE selects
// (aqz_handoff.hh: round robin over the visible devices by default, one
// stream per GPU); nullptr -- no device, AQZ_DEVICE=off, not multiscale --
// keeps the reference's CPU path.  AQZ_Z_SLABS=N splits a volume stream
// (a z Space dimension before y, acquisition storage order) into N z slabs
// on the next N selected devices (BASELINE configs[3]: 4 GPUs).
inline std::unique_ptr<GpuMultiscaleArrayBase>
make_gpu_multiscale_array(std::shared_ptr<ArrayConfig> config,
                          std::shared_ptr<ThreadPool> thread_pool,
                          std::shared_ptr<FileHandlePool> file_handle_pool,
                          std::shared_ptr<S3ConnectionPool> s3_connection_pool,
                          const ZarrArraySettings& settings)
{
    if (!settings.multiscale || !config->downsampling_method)
        return nullptr;
    int32_t n = 0;
    if (aqz_device_count(&n) != AQZ_STATUS_SUCCESS)
        return nullptr;
    const aqz_binding::SlabPlan plan = gpu_slab_plan(settings);
    std::vector<int32_t> devices;
    for (size_t r = 0; r < std::max<size_t>(1, plan.begin.size()); ++r) {
        const int32_t device = aqz_binding::select_device(n);
        if (device < 0)
            return nullptr;
        devices.push_back(device);
    }
    return std::make_unique<GpuMultiscaleArray>(config, thread_pool, file_handle_pool,
                                                s3_connection_pool, settings, devices, plan);
}

} // namespace zarr
