// binding_doubles.hh -- TEST INFRASTRUCTURE ONLY (never part of the product).
//
// Test doubles for the three reference classes the drop-in binding
// (integration/multiscale.array.gpu.cpp) derives from or writes to, whose
// definitions do not build from this image: zarr::Array (array.cpp needs
// crc32c), zarr::MultiscaleArray (multiscale.array.cpp needs array.base.cpp,
// which needs a newer nlohmann than the image's) and zarr::Shard (shard.cpp
// needs crc32c and the sinks; sink.cpp needs minio-cpp, an empty submodule).
// They are NOT the reference and not stand-ins for it in a reference build:
// they are this repo's own classes, named ArrayDouble / MultiscaleArrayDouble
// / ShardDouble, which the binding's code is compiled against (its
// GpuArrayBase / GpuMultiscaleArrayBase aliases, AQZ_BINDING_TEST_BASES) so
// that the binding's own code runs on the GPU.  Each member the binding
// touches is restated from the reference, cited file:line, and every place
// where the reference would silently do the wrong thing with what the
// binding hands it (a chunk written twice, a write after a shard was
// finalized, close_ finding bytes it would flush from CPU chunk buffers that
// the GPU path never fills) is recorded as an error instead.
//
// Everything else the binding uses is the reference itself, compiled from
// /root/reference by oracle/Makefile (target `binding`): ArrayConfig
// (array.base.hh, inline), ArrayDimensions, Downsampler (writer
// configurations), ThreadPool, the logger and zarr.common's helpers.
#pragma once

#define AQZ_BINDING_TEST_BASES 1

#include "array.hh"
#include "downsampler.hh"
#include "macros.hh"
#include "multiscale.array.hh"
#include "zarr.common.hh"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace zarr {

// What the doubles saw, read by the harness after close.
struct BindingLog
{
    struct Chunk
    {
        uint32_t level, append, shard, internal;
        bool skipped;
        std::vector<uint8_t> bytes; // empty unless keep_bytes
        uint64_t nbytes;
    };
    struct ShardEnd
    {
        uint32_t level, append, shard;
        bool complete;     // every internal index written or skipped
        bool by_countdown; // finalized by its last writer (shard.cpp:97-104)
    };
    struct LevelEnd
    {
        uint64_t frames_written = 0, total_bytes_written = 0, last_frame_id = 0;
        uint64_t bytes_to_flush = 0, metadata_writes = 0;
        uint32_t flushed_band_count = 0, append_chunk_index = 0, current_layer = 0;
        std::vector<uint64_t> rollovers; // frames_written_() at each rollover_
        bool closed = false;
    };

    std::mutex mu;
    std::vector<Chunk> chunks;
    std::vector<ShardEnd> shard_ends;
    std::map<uint32_t, LevelEnd> levels;
    std::vector<std::string> errors;
    bool keep_bytes = true; // false: a timing run, sizes only

    void error(const std::string& e)
    {
        std::lock_guard lk(mu);
        errors.push_back(e);
    }
};

inline BindingLog&
binding_log()
{
    static BindingLog log;
    return log;
}

struct ShardDoubleConfig
{
    std::string path;
    size_t chunks_per_shard;
    size_t bytes_per_chunk;
    uint32_t level, append, shard;
};

// zarr::Shard (shard.hh:25-75, shard.cpp:13-190): a countdown over the
// shard's internal indices -- each written (write_chunk) or skipped
// (skip_chunk) once; the last one writes the index table and finalizes the
// shard; a trailing partial shard is finalized at close (finalize()).  The
// sink is the log: the bytes Shard::write_chunk would put at the claimed
// offset are recorded with the shard's coordinates.
class ShardDouble
{
  public:
    static constexpr uint64_t kUnwritten = ~uint64_t(0); // kUnwrittenSentinel

    explicit ShardDouble(const ShardDoubleConfig& cfg)
      : cfg_(cfg)
      , offsets_(cfg.chunks_per_shard, kUnwritten)
      , extents_(cfg.chunks_per_shard, kUnwritten)
      , touched_(cfg.chunks_per_shard, 0)
      , unwritten_(cfg.chunks_per_shard)
    {
    }

    // shard.cpp:36-52: a shard dropped without its countdown completing or
    // finalize() (an aborted stream) is finalized here
    ~ShardDouble()
    {
        std::unique_lock lk(mu_);
        if (!finalized_)
            finalize_unlocked_(false);
    }

    // shard.cpp:54-109
    [[nodiscard]] bool write_chunk(uint32_t internal, const std::vector<uint8_t>& buffer)
    {
        EXPECT(internal < offsets_.size(), "Internal index ", internal, " out of bounds");
        {
            std::unique_lock lk(mu_);
            if (finalized_) {
                // the reference returns the cached result: the chunk is lost
                binding_log().error(where_(internal) + ": written after its shard was finalized");
                return finalize_ok_;
            }
            if (touched_[internal]++) {
                // the fake sink never fails, so nothing here is a retry
                binding_log().error(where_(internal) + ": written or skipped twice");
                return false;
            }
            extents_[internal] = buffer.size();
            offsets_[internal] = file_offset_;
            file_offset_ += buffer.size();
        }
        {
            std::lock_guard lk(binding_log().mu);
            BindingLog& log = binding_log();
            log.chunks.push_back(BindingLog::Chunk{
              cfg_.level, cfg_.append, cfg_.shard, internal, false,
              log.keep_bytes ? buffer : std::vector<uint8_t>{}, buffer.size() });
        }
        return count_down_();
    }

    // shard.cpp:111-134
    [[nodiscard]] bool skip_chunk(uint32_t internal)
    {
        EXPECT(internal < offsets_.size(), "Internal index ", internal, " out of bounds");
        {
            std::unique_lock lk(mu_);
            if (finalized_) {
                binding_log().error(where_(internal) + ": skipped after its shard was finalized");
                return finalize_ok_;
            }
            if (touched_[internal]++) {
                binding_log().error(where_(internal) + ": written or skipped twice");
                return false;
            }
            offsets_[internal] = kUnwritten;
            extents_[internal] = kUnwritten;
        }
        {
            std::lock_guard lk(binding_log().mu);
            binding_log().chunks.push_back(
              BindingLog::Chunk{ cfg_.level, cfg_.append, cfg_.shard, internal, true, {}, 0 });
        }
        return count_down_();
    }

    // shard.cpp:168-173: finalize at close (a trailing partial shard)
    [[nodiscard]] bool finalize()
    {
        std::unique_lock lk(mu_);
        return finalize_unlocked_(false);
    }

    const std::string& path() const { return cfg_.path; }

  private:
    ShardDoubleConfig cfg_;
    std::vector<uint64_t> offsets_, extents_;
    std::vector<uint8_t> touched_;
    std::atomic<uint64_t> unwritten_;
    uint64_t file_offset_ = 0;
    bool finalized_ = false, finalize_ok_ = false;
    std::mutex mu_;

    std::string where_(uint32_t internal) const
    {
        return "level " + std::to_string(cfg_.level) + " append " + std::to_string(cfg_.append) +
               " shard " + std::to_string(cfg_.shard) + " internal " + std::to_string(internal);
    }

    bool count_down_()
    {
        CHECK(unwritten_ > 0);
        if (unwritten_.fetch_sub(1) == 1) {
            std::unique_lock lk(mu_);
            return finalize_unlocked_(true);
        }
        return true;
    }

    // finalize_unlocked_ (shard.cpp:175-): write_table_ (:146-166) and flush: the table is the offsets
    // and extents; here the shard's end state is recorded instead
    bool finalize_unlocked_(bool by_countdown)
    {
        if (finalized_)
            return finalize_ok_;
        finalized_ = true;
        finalize_ok_ = true;
        std::lock_guard lk(binding_log().mu);
        binding_log().shard_ends.push_back(BindingLog::ShardEnd{
          cfg_.level, cfg_.append, cfg_.shard, unwritten_.load() == 0, by_countdown });
        return true;
    }
};

class MultiscaleArrayDouble;

// zarr::Array (array.hh:12-104) as far as GpuArray reaches into it.
class ArrayDouble
{
  public:
    // array.cpp:87-137 (and ArrayBase's, array.base.cpp:8-22)
    ArrayDouble(std::shared_ptr<ArrayConfig> config,
                std::shared_ptr<ThreadPool> thread_pool,
                std::shared_ptr<FileHandlePool> file_handle_pool,
                std::shared_ptr<S3ConnectionPool> s3_connection_pool)
      : config_(config)
      , thread_pool_(thread_pool)
      , s3_connection_pool_(s3_connection_pool)
      , file_handle_pool_(file_handle_pool)
      , write_counter_{ 0 }
      , max_bytes_(config->dimensions->max_byte_count())
      , bytes_per_frame_(bytes_of_frame(*config->dimensions, config->dtype))
      , total_bytes_written_{ 0 }
      , bytes_to_flush_{ 0 }
      , append_chunk_index_{ 0 }
      , is_closing_{ false }
      , last_successful_frame_id_{ 0 }
      , current_layer_{ 0 }
      , flushed_band_count_{ 0 }
    {
        CHECK(config_);
        CHECK(thread_pool_);
        EXPECT(config_->dimensions->number_of_chunks_in_memory() > 0,
               "Array has zero chunks in memory");
        data_root_ = config_->dimensions->is_2d()
                       ? node_path_() + "/c"
                       : node_path_() + "/c/" + std::to_string(append_chunk_index_);
    }
    virtual ~ArrayDouble() = default;

    // array.cpp:139-151: the CPU chunk buffers, allocated lazily by
    // write_frame_to_chunks_ -- which GpuArray never runs
    virtual size_t memory_usage() const noexcept { return 0; }

    // the CPU path: must not run under the binding
    [[nodiscard]] virtual WriteResult write_frame(std::vector<uint8_t>&,
                                                  size_t& bytes_written,
                                                  uint64_t)
    {
        bytes_written = 0;
        binding_log().error("Array::write_frame (the CPU path) was called");
        return WriteResult::OutOfBounds;
    }

    // array.cpp:226-229
    size_t max_bytes() const { return max_bytes_; }

  protected:
    std::shared_ptr<ArrayConfig> config_;
    std::shared_ptr<ThreadPool> thread_pool_;
    std::shared_ptr<S3ConnectionPool> s3_connection_pool_;
    std::shared_ptr<FileHandlePool> file_handle_pool_;

    std::vector<std::shared_ptr<ShardDouble>> shards_;
    std::mutex shards_mutex_;

    std::atomic<size_t> write_counter_;
    std::mutex write_counter_mutex_;
    std::condition_variable write_counter_cv_;

    std::vector<std::string> data_paths_;

    const uint64_t max_bytes_;
    const uint64_t bytes_per_frame_;
    uint64_t total_bytes_written_;
    uint64_t bytes_to_flush_;
    uint32_t append_chunk_index_;
    std::string data_root_;
    bool is_closing_;

    uint64_t last_successful_frame_id_;
    uint32_t current_layer_;

    uint32_t flushed_band_count_;

    std::vector<uint64_t> rollovers_;
    uint64_t metadata_writes_ = 0;

    uint32_t level_() const { return config_->level_of_detail; }

    // array.base.cpp:61-70
    std::string node_path_() const
    {
        std::string key = config_->store_root;
        if (!config_->node_key.empty())
            key += "/" + config_->node_key;
        return key;
    }

    // array.base.cpp:94-: the array's zarr.json (its shape follows
    // frames_written_); counted here
    [[nodiscard]] bool write_metadata_()
    {
        ++metadata_writes_;
        return true;
    }

    // array.cpp:433-461 (construct_data_paths, sink.cpp:48-, names the
    // shard files under data_root_; here a label per shard)
    void make_shards_()
    {
        if (!data_paths_.empty())
            return;
        const auto& dims = config_->dimensions;
        const size_t n_shards = dims->number_of_shards();
        for (size_t s = 0; s < n_shards; ++s)
            data_paths_.push_back(data_root_ + "/shard" + std::to_string(s));
        std::unique_lock lock(shards_mutex_);
        shards_.resize(n_shards);
        for (size_t s = 0; s < n_shards; ++s)
            shards_[s] = std::make_shared<ShardDouble>(ShardDoubleConfig{
              data_paths_[s], dims->chunks_per_shard(), dims->bytes_per_chunk(), level_(),
              append_chunk_index_, uint32_t(s) });
    }

    // array.cpp:924-937
    bool should_rollover_() const
    {
        const auto& dims = config_->dimensions;
        const auto& append_dim = dims->final_dim();
        size_t frames_before_flush = append_dim.chunk_size_px * append_dim.shard_size_chunks;
        for (size_t i = 1; i < dims->ndims() - 2; ++i)
            frames_before_flush *= dims->at(i).array_size_px;
        CHECK(frames_before_flush > 0);
        return frames_written_() % frames_before_flush == 0;
    }

    // array.cpp:625-662
    void dispatch_skip_job_(std::shared_ptr<ShardDouble> shard,
                            uint32_t internal_idx,
                            uint32_t shard_idx)
    {
        write_counter_.fetch_add(1);
        write_counter_cv_.notify_all();
        auto job = [this, shard, internal_idx, shard_idx](std::string& err) {
            ThreadPool::TaskResult result;
            try {
                if (shard->skip_chunk(internal_idx)) {
                    result = ThreadPool::TaskResult::Success;
                } else {
                    err = "Failed to skip chunk " + std::to_string(internal_idx) + " of shard " +
                          std::to_string(shard_idx);
                    result = ThreadPool::TaskResult::Fatal;
                }
            } catch (const std::exception& exc) {
                err = std::string("Failed skipping chunk: ") + exc.what();
                result = ThreadPool::TaskResult::Fatal;
            }
            write_counter_.fetch_sub(1);
            write_counter_cv_.notify_all();
            return result;
        };
        if (thread_pool_->n_threads() == 1 || !thread_pool_->push_job(job)) {
            if (!thread_pool_->execute_job(std::move(job)))
                LOG_ERROR("Failed to skip chunk ", internal_idx, " of shard ", shard_idx);
        }
    }

    // array.cpp:939-951
    void rollover_()
    {
        rollovers_.push_back(frames_written_());
        close_sinks_();
        ++append_chunk_index_;
        data_root_ = config_->dimensions->is_2d()
                       ? node_path_() + "/c"
                       : node_path_() + "/c/" + std::to_string(append_chunk_index_);
    }

    // array.cpp:967-971
    void close_sinks_()
    {
        data_paths_.clear();
        shards_.clear();
    }

    // array.cpp:954-964
    [[nodiscard]] bool finalize_shards_()
    {
        std::unique_lock lock(shards_mutex_);
        bool ok = true;
        for (auto& shard : shards_)
            if (shard && !shard->finalize())
                ok = false;
        return ok;
    }

    // array.cpp:974-977
    size_t frames_written_() const { return total_bytes_written_ / bytes_per_frame_; }

    // array.cpp:375-424.  bytes_to_flush_ > 0 here would make the reference
    // flush the open layer (compress_and_flush_data_ / flush_layer_remainder_)
    // from its CPU chunk buffers, which the GPU path never fills: an error.
    [[nodiscard]] virtual bool close_()
    {
        is_closing_ = true;
        if (bytes_to_flush_ > 0)
            binding_log().error("level " + std::to_string(level_()) + ": close_ finds " +
                                std::to_string(bytes_to_flush_) +
                                " bytes to flush from CPU chunk buffers");
        {
            // the reference waits with the predicate (array.cpp:390-392) and
            // would block forever on a lost wake-up (a job that decremented
            // without the mutex between the check and the wait); here a
            // timed wait that then finds the counter at 0 records that
            // instead of hanging
            std::unique_lock lock(write_counter_mutex_);
            while (write_counter_.load() != 0) {
                if (write_counter_cv_.wait_for(lock, std::chrono::seconds(5)) ==
                      std::cv_status::timeout &&
                    write_counter_.load() == 0)
                    binding_log().error("level " + std::to_string(level_()) +
                                        ": close_ missed the writer jobs' last "
                                        "notification (a lost wake-up)");
            }
        }
        bool ok = finalize_shards_();
        close_sinks_();
        if (frames_written_() > 0)
            ok = write_metadata_() && ok;
        BindingLog::LevelEnd e;
        e.frames_written = frames_written_();
        e.total_bytes_written = total_bytes_written_;
        e.last_frame_id = last_successful_frame_id_;
        e.bytes_to_flush = bytes_to_flush_;
        e.metadata_writes = metadata_writes_;
        e.flushed_band_count = flushed_band_count_;
        e.append_chunk_index = append_chunk_index_;
        e.current_layer = current_layer_;
        e.rollovers = rollovers_;
        e.closed = ok;
        {
            std::lock_guard lk(binding_log().mu);
            binding_log().levels[level_()] = std::move(e);
        }
        is_closing_ = false;
        return ok;
    }

    friend class MultiscaleArrayDouble;
};

// zarr::MultiscaleArray (multiscale.array.hh:9-65) as far as
// GpuMultiscaleArray reaches into it.
class MultiscaleArrayDouble
{
  public:
    // multiscale.array.cpp:24-44, with create_downsampler_ (:173-190,
    // make_base_array_config_ :278-289) and create_arrays_ (:138-160) --
    // the reference's own Downsampler, an ArrayDouble per writer
    // configuration
    MultiscaleArrayDouble(std::shared_ptr<ArrayConfig> config,
                          std::shared_ptr<ThreadPool> thread_pool,
                          std::shared_ptr<FileHandlePool> file_handle_pool,
                          std::shared_ptr<S3ConnectionPool> s3_connection_pool)
      : config_(config)
      , thread_pool_(thread_pool)
      , s3_connection_pool_(s3_connection_pool)
      , file_handle_pool_(file_handle_pool)
    {
        CHECK(config_);
        CHECK(thread_pool_);
        bytes_per_frame_ =
          config_->dimensions == nullptr ? 0 : bytes_of_frame(*config_->dimensions, config_->dtype);
        if (config_->downsampling_method) {
            auto base = std::make_shared<ArrayConfig>(
              config_->store_root, config_->node_key + "/0", config_->bucket_name,
              config_->compression_params, config_->dimensions, config_->dtype, std::nullopt, 0,
              config_->max_levels);
            downsampler_ = std::make_unique<Downsampler>(base, *config_->downsampling_method);
            const auto& configs = downsampler_->writer_configurations();
            arrays_.resize(configs.size());
            for (const auto& [lod, cfg] : configs)
                arrays_[lod] = std::make_unique<ArrayDouble>(cfg, thread_pool_,
                                                             file_handle_pool_,
                                                             s3_connection_pool_);
        }
        array_frame_ids_.resize(arrays_.size(), 0);
        EXPECT(!arrays_.empty(), "No Arrays created!");
    }
    virtual ~MultiscaleArrayDouble() = default;

    // multiscale.array.cpp:47-55
    virtual size_t memory_usage() const noexcept
    {
        size_t total = 0;
        for (const auto& a : arrays_)
            total += a->memory_usage();
        return total;
    }

    // the CPU path (multiscale.array.cpp:58-74): must not run
    [[nodiscard]] virtual WriteResult write_frame(std::vector<uint8_t>&,
                                                  size_t& bytes_written,
                                                  uint64_t)
    {
        bytes_written = 0;
        binding_log().error("MultiscaleArray::write_frame (the CPU path) was called");
        return WriteResult::OutOfBounds;
    }

    // multiscale.array.cpp:77-80
    size_t max_bytes() const { return arrays_[0]->max_bytes(); }

    // finalize_array (array.base.cpp): close_ through the base
    [[nodiscard]] bool finalize() { return close_(); }

    uint64_t group_metadata_writes() const { return metadata_writes_; }

  protected:
    std::shared_ptr<ArrayConfig> config_;
    std::shared_ptr<ThreadPool> thread_pool_;
    std::shared_ptr<S3ConnectionPool> s3_connection_pool_;
    std::shared_ptr<FileHandlePool> file_handle_pool_;

    std::unique_ptr<Downsampler> downsampler_;
    std::vector<std::unique_ptr<ArrayDouble>> arrays_;
    std::vector<uint64_t> array_frame_ids_;

    size_t bytes_per_frame_ = 0;
    uint64_t metadata_writes_ = 0;

    // multiscale.array.cpp:113-135
    [[nodiscard]] virtual bool close_()
    {
        for (auto& a : arrays_)
            if (!a->close_()) {
                LOG_ERROR("Error closing group: failed to finalize sub-array");
                return false;
            }
        ++metadata_writes_;
        arrays_.clear();
        return true;
    }
};

using GpuArrayBase = ArrayDouble;
using GpuMultiscaleArrayBase = MultiscaleArrayDouble;

} // namespace zarr
