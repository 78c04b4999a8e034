// multiscale.array.gpu.cpp -- the reference-side binding of the MI355X stage.
//
// This is the file a maintainer adds to acquire-zarr's src/streaming/ (built
// when ZARR_WITH_AQZ is on).  It is complete: the
// CPU suite compiles it with -fsyntax-only against the reference's own
// headers (tests/test_abi_pin_cpu.py), so every member it touches exists
// with the type used here.
//
//   GpuArray            : zarr::Array (array.hh:12-104) that accepts chunk
//                         layers (or dim-1 bands) filled on the GPU instead
//                         of running write_frame_to_chunks_ (array.cpp:
//                         507-622), then runs the reference's own flush /
//                         rollover / band logic (array.cpp:196-219, 762-908).
//   GpuMultiscaleArray  : zarr::MultiscaleArray (multiscale.array.hh:9-65)
//                         whose write_frame (multiscale.array.cpp:57-74)
//                         appends frames to the aqz stage -- level-0 tile
//                         split, Downsampler::add_frame and every level's
//                         tile split on the device -- and hands completed
//                         layers to the per-level GpuArrays through the
//                         asynchronous hand-off of aqz_handoff.hh.  Metadata
//                         (zarr.json, OME multiscales) stays the reference's:
//                         the base class keeps its Downsampler for level
//                         geometry and get_metadata(), which aqz reproduces
//                         byte for byte.
//
// ZarrStream_s::configure_array_ (zarr.stream.cpp:1231-1279) constructs a
// GpuMultiscaleArray instead of zarr::make_array's MultiscaleArray when the
// array is multiscale and a device is present.
#include "array.hh"
#include "macros.hh"
#include "multiscale.array.hh"
#include "zarr.common.hh"

#include "aqz_gpu.h"
#include "aqz_handoff.hh"

#include <memory>
#include <vector>

namespace zarr {

class GpuArray final : public Array
{
  public:
    using Array::Array;

    // Chunk slots [c0, c0 + n) of the current layer from a handed-off
    // buffer (n chunks of bytes_per_chunk) and their has_data bytes.  An
    // all-zero chunk keeps an empty slot, which dispatch_chunk_job_ skips
    // exactly like a chunk whose has_data is false (array.cpp:713-720).
    void install_chunks(const uint8_t* chunks, const uint8_t* has_data, uint32_t c0,
                        uint32_t n)
    {
        const size_t bpc = config_->dimensions->bytes_per_chunk();
        const size_t bpp = bytes_of_type(config_->dtype);
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t c = c0 + i;
            std::unique_lock lock(chunk_mutexes_[c]);
            if (!has_data[i]) {
                chunks_[c].reset();
                continue;
            }
            auto chunk = std::make_shared<Chunk>(bpc, bpp);
            // one "row" of the whole chunk: Chunk's only writer
            chunk->write_tile_rows(0, chunks + size_t(i) * bpc, bpc, bpc, bpc, 1);
            chunks_[c] = std::move(chunk);
        }
    }

    // `frames` more frames are in the chunk buffers: the tail of
    // Array::write_frame after write_frame_to_chunks_ (array.cpp:196-219).
    // flush = false only for the zero-filled partial last layer, which
    // Array::close_ flushes (array.cpp:380-387).
    WriteResult commit_frames(uint64_t frames, bool flush = true)
    {
        const uint64_t nbytes = frames * bytes_per_frame_;
        if (max_bytes_ > 0 && total_bytes_written_ + nbytes > max_bytes_)
            return WriteResult::OutOfBounds;
        last_successful_frame_id_ = frames_written_() + frames - 1;
        bytes_to_flush_ += nbytes;
        total_bytes_written_ += nbytes;
        if (!flush)
            return WriteResult::Ok;
        if (config_->dimensions->supports_dim1_banding()) {
            CHECK(flush_completed_bands_());
        } else if (should_flush_()) {
            CHECK(compress_and_flush_data_());
            if (should_rollover_()) {
                rollover_();
                CHECK(write_metadata_());
            }
            bytes_to_flush_ = 0;
        }
        return WriteResult::Ok;
    }

    bool close_array() { return close_(); }
};

class GpuMultiscaleArray final
  : public MultiscaleArray
  , private aqz_binding::HandoffSink
{
  public:
    // settings: the ZarrArraySettings the stream was configured with
    // (acquisition-order dims + storage order, zarr.types.h:157-169).
    GpuMultiscaleArray(std::shared_ptr<ArrayConfig> config,
                       std::shared_ptr<ThreadPool> thread_pool,
                       std::shared_ptr<FileHandlePool> file_handle_pool,
                       std::shared_ptr<S3ConnectionPool> s3_connection_pool,
                       const ZarrArraySettings& settings,
                       int device,
                       uint32_t batch_frames = 64,
                       uint32_t host_slots = 2)
      : MultiscaleArray(config, thread_pool, file_handle_pool, s3_connection_pool)
    {
        EXPECT(downsampler_ != nullptr, "GpuMultiscaleArray needs a downsampling method");
        // per-level writers that take GPU-filled layers (create_arrays_,
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
                             device };
        aqz_stage_options opt{};
        opt.max_batch_frames = batch_frames;
        opt.layer_slots = 2;
        EXPECT(aqz_stage_create(&desc, &opt, &stage_) == AQZ_STATUS_SUCCESS,
               "aqz_stage_create failed");
        EXPECT(aqz_stage_n_levels(stage_) == arrays_.size(),
               "level count differs from the Downsampler's");
        aqz_binding::HandoffSink& sink = *this;
        handoff_ = std::make_unique<aqz_binding::Handoff>(stage_, bytes_per_frame_,
                                                          batch_frames, host_slots, sink);
        EXPECT(handoff_->status() == AQZ_STATUS_SUCCESS, "aqz hand-off buffers: ",
               aqz_status_message(handoff_->status()));
    }

    ~GpuMultiscaleArray() override
    {
        handoff_.reset();
        aqz_stage_destroy(stage_);
    }

    size_t memory_usage() const noexcept override
    {
        aqz_memory_usage m{};
        (void)aqz_stage_memory_usage(stage_, &m);
        return MultiscaleArray::memory_usage() + m.pinned_bytes + handoff_->host_bytes();
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
        EXPECT(s == AQZ_STATUS_SUCCESS, "aqz stage: ", aqz_status_message(s));
        bytes_written = frame.size();
        return WriteResult::Ok;
    }

  protected:
    bool close_() override
    {
        try {
            const aqz_status s = handoff_->close();
            EXPECT(s == AQZ_STATUS_SUCCESS, "aqz stage: ", aqz_status_message(s));
        } catch (const std::exception& exc) {
            LOG_ERROR("Failed to finalize the GPU stage: ", exc.what());
            return false;
        }
        return MultiscaleArray::close_();
    }

  private:
    // aqz_binding::HandoffSink: units land in frame order per level
    void install(uint32_t level, const uint8_t* chunks, const uint8_t* has_data, uint32_t c0,
                 uint32_t n) override
    {
        gpu_arrays_[level]->install_chunks(chunks, has_data, c0, n);
    }

    aqz_status commit(uint32_t level, uint64_t frames, bool flush) override
    {
        return gpu_arrays_[level]->commit_frames(frames, flush) == WriteResult::Ok
                 ? AQZ_STATUS_SUCCESS
                 : AQZ_STATUS_WRITE_OUT_OF_BOUNDS;
    }

    aqz_stage* stage_ = nullptr;
    std::vector<aqz_dimension> dims_;
    std::vector<GpuArray*> gpu_arrays_;
    std::unique_ptr<aqz_binding::Handoff> handoff_;
};

} // namespace zarr
