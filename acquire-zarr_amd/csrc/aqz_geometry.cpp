// aqz_geometry.cpp -- see aqz_geometry.hh.  Citations are to
// /root/reference/src/streaming/.
#include "aqz_geometry.hh"

#include <algorithm>
#include <bit>

namespace aqz {

size_t
bytes_of_type(int32_t dtype)
{
    // zarr.common.cpp:47-70
    switch (dtype) {
        case 0: // uint8
        case 4: // int8
            return 1;
        case 1:
        case 5:
            return 2;
        case 2:
        case 6:
        case 8:
            return 4;
        case 3:
        case 7:
        case 9:
            return 8;
        default:
            throw Error(1, "Invalid data type: " + std::to_string(dtype));
    }
}

ArrayDimensions::ArrayDimensions(std::vector<Dim> dims,
                                 int32_t dtype,
                                 const std::vector<size_t>& order)
  : is_2d_(dims.size() == 2)
  , dtype_(dtype)
  , bytes_per_chunk_(bytes_of_type(dtype))
{
    if (dims.size() < 2)
        throw Error(9, "Array must have at least two dimensions.");
    // 2-D arrays get a phantom singleton (array.dimensions.cpp:149-153)
    std::vector<size_t> ord = order;
    if (is_2d_) {
        dims.insert(dims.begin(), Dim{ kOther, 1, 1, 1 });
        if (!ord.empty()) {
            for (auto& o : ord)
                ++o;
            ord.insert(ord.begin(), 0);
        }
    }
    const size_t n = dims.size();
    if (dims[n - 2].type != kSpace || dims[n - 1].type != kSpace)
        throw Error(9, "Last two dimensions must be spatial");
    for (const auto& d : dims)
        if (d.chunk_size_px == 0)
            throw Error(9, "chunk_size_px must be > 0");

    // compute_transposition (array.dimensions.cpp:9-135)
    dims_ = dims;
    if (!ord.empty()) {
        if (ord.size() != n)
            throw Error(9, "storage_dimension_order has wrong length");
        if (ord[0] != 0)
            throw Error(9, "dimension 0 must stay first in storage order");
        std::vector<size_t> a2s(n), s2a(n);
        std::vector<bool> seen(n, false);
        std::vector<Dim> sdims(n);
        for (size_t s = 0; s < n; ++s) {
            const size_t a = ord[s];
            if (a >= n || seen[a])
                throw Error(9, "invalid storage_dimension_order");
            seen[a] = true;
            sdims[s] = dims[a];
            a2s[a] = s;
            s2a[s] = a;
        }
        if (sdims[n - 2].type != kSpace || sdims[n - 1].type != kSpace)
            throw Error(9, "After reordering, last two dims must be spatial");
        bool identity = true;
        for (size_t i = 0; i < n; ++i)
            identity &= a2s[i] == i;
        dims_ = sdims;
        if (!identity) {
            transposed_ = true;
            acq_to_storage_ = a2s;
            acq_dims_ = dims;
            const bool dim0_unbounded = dims[0].array_size_px == 0;
            const size_t start = dim0_unbounded ? 1 : 0;
            const size_t frame_dims = n - 2;
            const size_t lookup_dims = frame_dims - start;
            uint64_t lookup_size = 1;
            for (size_t i = start; i < n - 2; ++i)
                lookup_size *= dims[i].array_size_px;
            frame_id_lookup_.resize(lookup_size);
            inner_frame_count_ = dim0_unbounded ? lookup_size : 0;
            std::vector<uint64_t> as(lookup_dims, 1), ss(lookup_dims, 1);
            for (size_t i = lookup_dims ? lookup_dims - 1 : 0; i > 0; --i) {
                const size_t di = start + i;
                as[i - 1] = as[i] * dims[di].array_size_px;
                ss[i - 1] = ss[i] * sdims[di].array_size_px;
            }
            std::vector<uint64_t> ac(lookup_dims), sc(lookup_dims);
            for (uint64_t f = 0; f < lookup_size; ++f) {
                uint64_t rem = f;
                for (size_t i = 0; i < lookup_dims; ++i) {
                    ac[i] = rem / as[i];
                    rem %= as[i];
                }
                for (size_t i = 0; i < lookup_dims; ++i)
                    sc[a2s[start + i] - start] = ac[i];
                uint64_t sf = 0;
                for (size_t i = 0; i < lookup_dims; ++i)
                    sf += sc[i] * ss[i];
                frame_id_lookup_[f] = sf;
            }
        }
    }

    // array.dimensions.cpp:168-178
    for (size_t i = 0; i < n; ++i) {
        bytes_per_chunk_ *= dims_[i].chunk_size_px;
        if (i > 0)
            chunks_in_memory_ *=
              parts_along(dims_[i].array_size_px, dims_[i].chunk_size_px);
    }
}

bool
ArrayDimensions::needs_xy_transposition() const
{
    // array.dimensions.cpp:562-575
    if (!transposed_)
        return false;
    const size_t n = ndims();
    return acq_to_storage_[n - 2] == n - 1 && acq_to_storage_[n - 1] == n - 2;
}

uint32_t
ArrayDimensions::chunk_lattice_index(uint64_t frame_id,
                                     uint32_t dim_index) const
{
    // array.dimensions.cpp:232-262
    const size_t n = ndims();
    if (dim_index >= n - 2)
        throw Error(3, "Invalid dimension index");
    if (dim_index == 0) {
        uint64_t divisor = dims_[0].chunk_size_px;
        for (size_t i = 1; i < n - 2; ++i)
            divisor *= dims_[i].array_size_px;
        return static_cast<uint32_t>(frame_id / divisor);
    }
    uint64_t mod_div = 1, div_div = 1;
    for (size_t i = dim_index; i < n - 2; ++i) {
        mod_div *= dims_[i].array_size_px;
        div_div *= (i == dim_index ? dims_[i].chunk_size_px
                                   : dims_[i].array_size_px);
    }
    return static_cast<uint32_t>((frame_id % mod_div) / div_div);
}

uint32_t
ArrayDimensions::tile_group_offset(uint64_t frame_id) const
{
    // array.dimensions.cpp:264-282
    const size_t n = ndims();
    std::vector<uint64_t> strides(n, 1);
    for (size_t i = n - 1; i > 0; --i)
        strides[i - 1] =
          strides[i] *
          parts_along(dims_[i].array_size_px, dims_[i].chunk_size_px);
    uint64_t offset = 0;
    for (size_t i = n - 3; i > 0; --i)
        offset += uint64_t(chunk_lattice_index(frame_id, i)) * strides[i];
    return static_cast<uint32_t>(offset);
}

uint64_t
ArrayDimensions::chunk_internal_offset(uint64_t frame_id) const
{
    // array.dimensions.cpp:284-314
    const size_t n = ndims();
    const uint64_t tile_size = bytes_of_type(dtype_) *
                               uint64_t(width_dim().chunk_size_px) *
                               height_dim().chunk_size_px;
    std::vector<uint64_t> as(n - 2, 1), cs(n - 2, 1);
    uint64_t offset = 0;
    for (int i = int(n) - 3; i > 0; --i) {
        const Dim& d = dims_[i];
        const uint64_t idx =
          (frame_id / as[i]) % d.array_size_px % d.chunk_size_px;
        as[i - 1] = as[i] * d.array_size_px;
        cs[i - 1] = cs[i] * d.chunk_size_px;
        offset += idx * cs[i];
    }
    offset += ((frame_id / as[0]) % dims_[0].chunk_size_px) * cs[0];
    return offset * tile_size;
}

uint64_t
ArrayDimensions::transpose_frame_id(uint64_t frame_id) const
{
    // array.dimensions.cpp:602-620
    if (!transposed_)
        return frame_id;
    if (inner_frame_count_ > 0) {
        const uint64_t outer = frame_id / inner_frame_count_;
        const uint64_t inner = frame_id % inner_frame_count_;
        return outer * inner_frame_count_ + frame_id_lookup_[inner];
    }
    return frame_id_lookup_.at(frame_id);
}

uint64_t
ArrayDimensions::frames_per_chunk_layer() const
{
    // array.dimensions.cpp:328-336
    uint64_t f = dims_[0].chunk_size_px;
    for (size_t i = 1; i + 2 < ndims(); ++i)
        f *= dims_[i].array_size_px;
    return f;
}

static uint32_t
shards_along(const Dim& d)
{
    // zarr.common.cpp:94-104
    if (d.shard_size_chunks == 0)
        return 0;
    return parts_along(parts_along(d.array_size_px, d.chunk_size_px),
                       d.shard_size_chunks);
}

uint32_t
ArrayDimensions::shard_index_for_chunk(uint32_t chunk_index) const
{
    // array.dimensions.cpp:461-502 (lattice index of dim 0 stays 0)
    const size_t n = ndims();
    std::vector<uint64_t> cs(n, 1);
    for (size_t i = n - 1; i > 0; --i)
        cs[i - 1] =
          cs[i] * parts_along(dims_[i].array_size_px, dims_[i].chunk_size_px);
    std::vector<uint32_t> lat(n, 0), ss(n, 1);
    for (size_t i = n - 1; i > 0; --i)
        lat[i] = static_cast<uint32_t>(chunk_index % cs[i - 1] / cs[i]);
    for (size_t i = n - 1; i > 0; --i)
        ss[i - 1] = ss[i] * shards_along(dims_[i]);
    uint32_t index = 0;
    for (size_t i = 0; i < n; ++i) {
        if (dims_[i].shard_size_chunks == 0)
            throw Error(1, "shard_size_chunks is 0");
        index += (lat[i] / dims_[i].shard_size_chunks) * ss[i];
    }
    return index;
}

uint32_t
ArrayDimensions::chunks_per_shard() const
{
    uint64_t n = 1;
    for (const Dim& d : dims_)
        n *= d.shard_size_chunks;
    if (n > 0xffffffffull)
        throw Error(1, "too many chunks per shard");
    return uint32_t(n);
}

uint32_t
ArrayDimensions::number_of_shards() const
{
    uint64_t n = 1;
    for (size_t i = 1; i < dims_.size(); ++i)
        n *= shards_along(dims_[i]);
    return uint32_t(n);
}

uint32_t
ArrayDimensions::shard_internal_index(uint32_t chunk_index) const
{
    // array.dimensions.cpp:504-548
    const size_t n = ndims();
    std::vector<uint64_t> cs(n, 1), lat(n, 0), is(n, 1);
    for (size_t i = n - 1; i > 0; --i)
        cs[i - 1] =
          cs[i] * parts_along(dims_[i].array_size_px, dims_[i].chunk_size_px);
    for (size_t i = n - 1; i > 0; --i)
        lat[i] = chunk_index % cs[i - 1] / cs[i];
    lat[0] = chunk_index / cs[0];
    for (size_t i = n - 1; i > 0; --i)
        is[i - 1] = is[i] * dims_[i].shard_size_chunks;
    uint64_t index = 0;
    for (size_t i = 0; i < n; ++i) {
        if (dims_[i].shard_size_chunks == 0)
            throw Error(1, "shard_size_chunks is 0");
        index += (lat[i] % dims_[i].shard_size_chunks) * is[i];
    }
    return static_cast<uint32_t>(index);
}

// array.dimensions.cpp:406-453: the chunks of layer `layer` (of one append-
// dimension shard row) that belong to `shard` fill some of its internal
// slots [layer * per_layer, (layer + 1) * per_layer); the rest is ragged
// padding.  Computed over the layer's own chunks (the reference filters the
// shard's whole chunk list by layer: the same set), ascending.
std::vector<uint32_t>
ArrayDimensions::skipped_internal_indices_for_shard_layer(uint32_t shard, uint32_t layer) const
{
    const uint32_t layers = std::max<uint32_t>(1, chunk_layers_per_shard());
    const uint32_t per_layer = chunks_per_shard() / layers;
    const uint64_t lo = uint64_t(layer) * per_layer;
    std::vector<uint8_t> filled(per_layer, 0);
    uint32_t n = 0;
    const uint32_t c0 = layer * chunks_in_memory_;
    for (uint32_t c = c0; c < c0 + chunks_in_memory_; ++c) {
        if (shard_index_for_chunk(c) != shard)
            continue;
        const uint64_t internal = shard_internal_index(c);
        if (internal >= lo && internal < lo + per_layer && !filled[internal - lo]) {
            filled[internal - lo] = 1;
            ++n;
        }
    }
    std::vector<uint32_t> out;
    if (n == per_layer)
        return out;
    for (uint32_t i = 0; i < per_layer; ++i)
        if (!filled[i])
            out.push_back(uint32_t(lo + i));
    return out;
}

// ---------------------------------------------------------------------------
// Pyramid level rule (downsampler.cpp:8-37, 494-597)
// ---------------------------------------------------------------------------
static Dim
downsample_dimension(const Dim& d)
{
    Dim o = d;
    o.array_size_px = (d.array_size_px + (d.array_size_px % 2)) / 2;
    const uint32_t n_chunks = parts_along(o.array_size_px, d.chunk_size_px);
    o.shard_size_chunks = std::min(n_chunks, d.shard_size_chunks);
    return o;
}

std::vector<std::vector<Dim>>
make_pyramid_levels(const std::vector<Dim>& dims,
                    uint32_t max_levels,
                    uint32_t force_levels)
{
    const size_t n = dims.size();
    if (n < 3)
        throw Error(1, "make_pyramid_levels needs >= 3 dims");
    const Dim& X = dims[n - 1];
    const Dim& Y = dims[n - 2];
    const Dim& Z = dims[n - 3];
    const uint32_t ncx = parts_along(X.array_size_px, X.chunk_size_px);
    const uint32_t nlx = ncx > 1 ? std::bit_width(ncx - 1) : 0;
    const uint32_t ncy = parts_along(Y.array_size_px, Y.chunk_size_px);
    const uint32_t nly = ncy > 1 ? std::bit_width(ncy - 1) : 0;
    uint32_t n_levels = std::min(nlx, nly);
    if (Z.type == kSpace) {
        const uint32_t ncz = parts_along(Z.array_size_px, Z.chunk_size_px);
        const uint32_t ndz = ncz > 1 ? std::bit_width(ncz - 1) : 0;
        n_levels = std::max(n_levels, ndz);
    }
    if (max_levels > 0)
        n_levels = std::min(n_levels, max_levels);
    if (force_levels > 0)
        n_levels = force_levels - 1;

    std::vector<std::vector<Dim>> levels{ dims };
    for (uint32_t level = 1; level <= n_levels; ++level) {
        const auto& prev = levels.back();
        std::vector<Dim> cur(prev.begin(), prev.end());
        const Dim& z = prev[n - 3];
        if (z.type == kSpace && z.array_size_px > z.chunk_size_px &&
            force_levels == 0)
            cur[n - 3] = downsample_dimension(z);
        const Dim& y = prev[n - 2];
        const Dim& x = prev[n - 1];
        const bool shrink =
          force_levels > 0
            ? std::min(y.array_size_px, x.array_size_px) > 1
            : std::min(y.array_size_px, x.array_size_px) >
                std::max(y.chunk_size_px, x.chunk_size_px);
        if (shrink) {
            cur[n - 2] = downsample_dimension(y);
            cur[n - 1] = downsample_dimension(x);
        }
        levels.push_back(std::move(cur));
    }
    return levels;
}

} // namespace aqz
