// aqz_geometry.hh -- host restatement of the reference's chunk-lattice and
// pyramid-level geometry.  It drives the device kernels' addressing (a table
// of per-frame chunk offsets per level) and is itself not a kernel.
//
//   ArrayDimensions      <- src/streaming/array.dimensions.{hh,cpp}
//   make_pyramid_levels  <- Downsampler::make_writer_configurations_
//                           (src/streaming/downsampler.cpp:494-597)
#pragma once

#include <cstddef>
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

namespace aqz {

enum DimType : int32_t
{
    kSpace = 0,
    kChannel = 1,
    kTime = 2,
    kOther = 3
};

struct Dim
{
    int32_t type{ kSpace };
    uint32_t array_size_px{ 0 };
    uint32_t chunk_size_px{ 0 };
    uint32_t shard_size_chunks{ 0 };
    bool operator==(const Dim& o) const
    {
        return type == o.type && array_size_px == o.array_size_px &&
               chunk_size_px == o.chunk_size_px &&
               shard_size_chunks == o.shard_size_chunks;
    }
};

// Thrown for invalid configuration; the C ABI maps it to a status code.
struct Error : std::runtime_error
{
    int32_t status;
    Error(int32_t s, const std::string& m)
      : std::runtime_error(m)
      , status(s)
    {
    }
};

size_t bytes_of_type(int32_t dtype);

inline uint32_t
parts_along(uint32_t array, uint32_t part)
{
    return (array + part - 1) / part;
}

// ArrayDimensions (array.dimensions.cpp:137-189).  dims are given in
// acquisition order; with a storage order the last two dims must stay
// spatial.  An XY swap (needs_xy_transposition) is rejected with
// NotYetImplemented by the GPU stage (frame transpose is a §8f "next" row).
class ArrayDimensions
{
  public:
    ArrayDimensions(std::vector<Dim> dims,
                    int32_t dtype,
                    const std::vector<size_t>& storage_order = {});

    size_t ndims() const { return dims_.size(); }
    const Dim& at(size_t i) const { return dims_.at(i); }
    const std::vector<Dim>& dims() const { return dims_; }
    const Dim& height_dim() const { return dims_[ndims() - 2]; }
    const Dim& width_dim() const { return dims_.back(); }
    int32_t dtype() const { return dtype_; }
    bool is_2d() const { return is_2d_; }

    uint32_t chunk_lattice_index(uint64_t frame_id, uint32_t dim_index) const;
    uint32_t tile_group_offset(uint64_t frame_id) const;
    uint64_t chunk_internal_offset(uint64_t frame_id) const;
    uint64_t transpose_frame_id(uint64_t frame_id) const;
    bool needs_transposition() const { return transposed_; }
    bool needs_xy_transposition() const;

    uint64_t bytes_per_chunk() const { return bytes_per_chunk_; }
    uint32_t number_of_chunks_in_memory() const { return chunks_in_memory_; }
    uint64_t frames_per_chunk_layer() const;
    uint32_t shard_index_for_chunk(uint32_t chunk_index) const;
    uint32_t shard_internal_index(uint32_t chunk_index) const;
    // array.dimensions.cpp:168-178, 376-397
    uint32_t chunks_per_shard() const;
    uint32_t number_of_shards() const;
    uint32_t chunk_layers_per_shard() const { return dims_[0].shard_size_chunks; }
    // Internal indices of shard `shard` that no chunk of chunk layer `layer`
    // (of one append-dimension shard row) fills -- the ragged padding the
    // reference skips so the shard's countdown completes
    // (array.dimensions.cpp:406-453)
    std::vector<uint32_t> skipped_internal_indices_for_shard_layer(uint32_t shard,
                                                                   uint32_t layer) const;
    // dim-1 banding (array.dimensions.cpp:344-373): append chunk 1 plus an
    // intermediate dim, no transposition; a band is one chunk row of dim 1
    bool supports_dim1_banding() const
    {
        return dims_[0].chunk_size_px == 1 && ndims() >= 4 && !transposed_;
    }
    uint32_t dim1_band_count() const
    {
        return parts_along(dims_[1].array_size_px, dims_[1].chunk_size_px);
    }
    uint64_t frames_per_dim1_band() const
    {
        uint64_t f = dims_[1].chunk_size_px;
        for (size_t i = 2; i + 2 < ndims(); ++i)
            f *= dims_[i].array_size_px;
        return f;
    }
    uint32_t chunks_per_dim1_band() const
    {
        return chunks_in_memory_ / dim1_band_count();
    }

  private:
    bool is_2d_;
    int32_t dtype_;
    std::vector<Dim> dims_; // storage order
    bool transposed_{ false };
    std::vector<size_t> acq_to_storage_;
    std::vector<Dim> acq_dims_;
    std::vector<uint64_t> frame_id_lookup_;
    uint64_t inner_frame_count_{ 0 };
    uint64_t bytes_per_chunk_;
    uint32_t chunks_in_memory_{ 1 };
};

// Level dims for a pyramid; level 0 = base.  dims are storage-order, with
// ndims >= 3 (the 2-D phantom already prepended).  force_levels > 0 is the
// bench extension of aqz_stage_options (keep halving XY).
std::vector<std::vector<Dim>>
make_pyramid_levels(const std::vector<Dim>& dims,
                    uint32_t max_levels,
                    uint32_t force_levels = 0);

} // namespace aqz
