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
//                         layers to the per-level GpuArrays.  Metadata
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

#include <cstring>
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

class GpuMultiscaleArray final : public MultiscaleArray
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
                       uint32_t batch_frames = 64)
      : MultiscaleArray(config, thread_pool, file_handle_pool, s3_connection_pool)
      , batch_(batch_frames)
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
        opt.max_batch_frames = batch_;
        opt.layer_slots = 2;
        EXPECT(aqz_stage_create(&desc, &opt, &stage_) == AQZ_STATUS_SUCCESS,
               "aqz_stage_create failed");
        const uint32_t nl = aqz_stage_n_levels(stage_);
        EXPECT(nl == arrays_.size(), "level count differs from the Downsampler's");
        levels_.resize(nl);
        for (uint32_t l = 0; l < nl; ++l) {
            Level& L = levels_[l];
            CHECK(aqz_stage_level_layout(stage_, l, &L.lay) == AQZ_STATUS_SUCCESS);
            int32_t banded = 0;
            CHECK(aqz_stage_band_geometry(stage_, l, &banded, &L.n_bands,
                                          &L.frames_per_band,
                                          &L.chunks_per_band) == AQZ_STATUS_SUCCESS);
            L.banded = banded != 0;
            const size_t nbytes = L.lay.bytes_per_chunk * L.chunks_per_band;
            CHECK(aqz_host_alloc(nbytes, reinterpret_cast<void**>(&L.chunks)) ==
                  AQZ_STATUS_SUCCESS);
            CHECK(aqz_host_alloc(L.chunks_per_band, reinterpret_cast<void**>(&L.has)) ==
                  AQZ_STATUS_SUCCESS);
        }
        CHECK(aqz_host_alloc(size_t(batch_) * bytes_per_frame_,
                             reinterpret_cast<void**>(&batch_buf_)) == AQZ_STATUS_SUCCESS);
    }

    ~GpuMultiscaleArray() override
    {
        for (Level& L : levels_) {
            aqz_host_free(L.chunks);
            aqz_host_free(L.has);
        }
        aqz_host_free(batch_buf_);
        aqz_stage_destroy(stage_);
    }

    size_t memory_usage() const noexcept override
    {
        aqz_memory_usage m{};
        (void)aqz_stage_memory_usage(stage_, &m);
        size_t staging = size_t(batch_) * bytes_per_frame_;
        for (const Level& L : levels_)
            staging += L.lay.bytes_per_chunk * L.chunks_per_band + L.chunks_per_band;
        return MultiscaleArray::memory_usage() + m.pinned_bytes + staging;
    }

    // MultiscaleArray::write_frame (multiscale.array.cpp:57-74) with the
    // checks of Array::write_frame (array.cpp:160-189).  Frames are
    // batched into pinned memory and appended `batch_` at a time.
    [[nodiscard]] WriteResult write_frame(std::vector<uint8_t>& frame,
                                          size_t& bytes_written,
                                          uint64_t frame_id) override
    {
        bytes_written = 0;
        if (frame.size() != bytes_per_frame_)
            return WriteResult::FrameSizeMismatch;
        if (frame_id != frames_accepted_)
            return WriteResult::FrameOutOfOrder;
        const uint64_t max = arrays_[0]->max_bytes();
        if (max > 0 && (frames_accepted_ + 1) * bytes_per_frame_ > max)
            return WriteResult::OutOfBounds;
        std::memcpy(batch_buf_ + size_t(n_batched_) * bytes_per_frame_, frame.data(),
                    bytes_per_frame_);
        ++n_batched_;
        ++frames_accepted_;
        if (n_batched_ == batch_) {
            const WriteResult r = append_batch_();
            if (r != WriteResult::Ok)
                return r;
        }
        bytes_written = frame.size();
        return WriteResult::Ok;
    }

  protected:
    bool close_() override
    {
        try {
            if (append_batch_() != WriteResult::Ok)
                return false;
            // zero-fill the partial last layer of every level (chunk.cpp:
            // 8-15) and hand it over unflushed; Array::close_ flushes it
            CHECK(aqz_stage_finalize(stage_) == AQZ_STATUS_SUCCESS);
            CHECK(hand_off_(true) == WriteResult::Ok);
        } catch (const std::exception& exc) {
            LOG_ERROR("Failed to finalize the GPU stage: ", exc.what());
            return false;
        }
        return MultiscaleArray::close_();
    }

  private:
    struct Level
    {
        aqz_level_layout lay{};
        bool banded = false;
        uint32_t n_bands = 1, chunks_per_band = 0;
        uint64_t frames_per_band = 0;
        uint64_t handed = 0; // frames of this level handed to its GpuArray
        uint8_t* chunks = nullptr;
        uint8_t* has = nullptr;
    };

    WriteResult append_batch_()
    {
        if (n_batched_ == 0)
            return WriteResult::Ok;
        const aqz_status s =
          aqz_stage_append(stage_, batch_buf_, n_batched_, AQZ_MEM_HOST_PINNED);
        if (s == AQZ_STATUS_WRITE_OUT_OF_BOUNDS)
            return WriteResult::OutOfBounds;
        EXPECT(s == AQZ_STATUS_SUCCESS, "aqz_stage_append: ", aqz_status_message(s));
        // the pinned batch is read asynchronously: reuse it once consumed
        while (aqz_stage_frames_consumed(stage_) < frames_accepted_)
            ;
        n_batched_ = 0;
        return hand_off_(false);
    }

    // Every complete unit (a dim-1 band where Array::flush_completed_bands_
    // applies, else a chunk layer) of every level goes D2H and into its
    // GpuArray, in frame order.  final: also the partial last unit.
    WriteResult hand_off_(bool final)
    {
        for (uint32_t l = 0; l < levels_.size(); ++l) {
            Level& L = levels_[l];
            const uint64_t written = aqz_stage_frames_written(stage_, l);
            const uint64_t unit = L.banded ? L.frames_per_band : L.lay.frames_per_layer;
            while (L.handed + unit <= written || (final && L.handed < written)) {
                const uint64_t layer = L.handed / L.lay.frames_per_layer;
                const uint32_t band =
                  L.banded ? uint32_t((L.handed % L.lay.frames_per_layer) / unit) : 0;
                const size_t nbytes = L.lay.bytes_per_chunk * L.chunks_per_band;
                if (L.banded)
                    CHECK(aqz_stage_copy_band_async(stage_, l, layer, band, L.chunks, nbytes,
                                                    L.has, L.chunks_per_band) ==
                          AQZ_STATUS_SUCCESS);
                else
                    CHECK(aqz_stage_copy_layer_async(stage_, l, layer, L.chunks, nbytes, L.has,
                                                     L.chunks_per_band) == AQZ_STATUS_SUCCESS);
                CHECK(aqz_stage_wait_copies(stage_) == AQZ_STATUS_SUCCESS);
                gpu_arrays_[l]->install_chunks(L.chunks, L.has, band * L.chunks_per_band,
                                               L.chunks_per_band);
                const uint64_t n = std::min(unit, written - L.handed);
                const WriteResult r = gpu_arrays_[l]->commit_frames(n, n == unit);
                if (r != WriteResult::Ok)
                    return r;
                L.handed += n;
            }
        }
        return WriteResult::Ok;
    }

    aqz_stage* stage_ = nullptr;
    std::vector<aqz_dimension> dims_;
    std::vector<GpuArray*> gpu_arrays_;
    std::vector<Level> levels_;
    const uint32_t batch_;
    uint8_t* batch_buf_ = nullptr;
    uint32_t n_batched_ = 0;
    uint64_t frames_accepted_ = 0;
};

} // namespace zarr
